"""Kernel stats of a c3 / c5 bench (tools/measure.sh steps c3prof / c5prof) -> markdown.

    python tools/size_md.py gpurun_out/<tag> <N> profiles/<name>.md

Reads <tag>/prof<N>/run_kernel_{stats,trace}.csv, the profiled bench line
<tag>/prof_bench<N>.json, the unprofiled <tag>/bench<N>.log and profiles/traffic_<N>.json.
Per-frame figures use the headline launches (largest grid per kernel, every launch of it):
a chunk of `frames_per_launch` frames runs as `streams_per_chunk` concurrent parts.
"""
import csv
import json
import os
import sys

src, n, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
pdir = os.path.join(src, f"prof{n}")
pb = json.loads(open(os.path.join(src, f"prof_bench{n}.json")).read().strip().splitlines()[-1])
bench = [l for l in open(os.path.join(src, f"bench{n}.log")) if l.startswith("{")][-1].strip()
chunk = pb["roofline"]["frames_per_launch"]
streams = pb["config"].get("streams_per_chunk", 1)
part = chunk / streams


def short(s):
    s = s.replace("HIP_vector_type<float, 2u>", "float2")
    s = s[5:] if s.startswith("void ") else s
    return s[:s.find("(")] if "(" in s else s


trace = [t for t in csv.DictReader(open(os.path.join(pdir, "run_kernel_trace.csv"))) if "fcdk::" in t["Kernel_Name"]]
by = {}
for t in trace:
    g = int(t["Grid_Size_X"]) * int(t["Grid_Size_Y"]) * int(t["Grid_Size_Z"])
    d = (int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e3
    by.setdefault(short(t["Kernel_Name"]), {}).setdefault(g, []).append(d)
traffic = {}
tp = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", f"traffic_{n}.json")
if os.path.exists(tp):
    traffic = json.load(open(tp))
cmd = pb["config"]["workload"]
lines = [f"# {os.path.basename(dst)[:-3]} — rocprofv3 --kernel-trace --stats, {n}x{n} frames (MI355X, 1 GPU)", "",
         f"Workload: {cmd}. Command: `rocprofv3 --kernel-trace --stats -f csv -- python3 bench.py --size {n} "
         f"--batch {pb['config']['batch_per_gpu']} --steps {pb['steps']} --warmup {pb['warmup']} --no-cpu-baseline` "
         f"(tools/measure.sh). Engine kernels only. Source: `{pdir}/`.", "",
         f"Largest-grid launches of each kernel (the throughput chain: {chunk:g}-frame chunks as {streams} concurrent "
         f"part(s) of {part:g} frames; the roofline pass's own single-stream launches of the demod kernels are in the "
         "same grid class and averaged in):", "",
         "| kernel | launches | avg us | us/frame (avg / frames per launch) |", "|---|---|---|---|"]
for k, g in sorted(by.items(), key=lambda kv: -sum(max(kv[1].items())[1])):
    grid, d = max(g.items())
    if len(d) < pb["steps"]:
        continue  # reference setup
    a = sum(d) / len(d)
    lines.append(f"| `{k}` | {len(d)} | {a:.1f} | {a / part:.2f} |")
lines += ["", "Stage split the bench reports (HIP events, us per frame): "
          + ", ".join(f"{k} {v}" for k, v in pb["stage_us_per_frame"].items()) + ".", ""]
if traffic:
    lines += [f"PMC traffic (`profiles/traffic_{n}.json`: FETCH_SIZE x2 / WRITE_SIZE x1 calibrated passes over "
              f"`bench.py --size {n} --batch {traffic['chunk']}`), MB per frame:", "",
              "| kernel | read | write | total |", "|---|---|---|---|"]
    for k, v in traffic["per_kernel"].items():
        f = v["frames_per_launch"]
        lines.append(f"| `{k}` | {v['read_bytes_per_launch'] / f / 1e6:.2f} | {v['write_bytes_per_launch'] / f / 1e6:.2f} | "
                     f"{v['bytes_per_frame'] / 1e6:.2f} |")
    lines += ["", f"Headline chain: {traffic['headline_bytes_per_frame'] / 1e6:.1f} MB per frame against "
              f"{traffic['headline_algorithmic_bytes_per_frame'] / 1e6:.1f} MB algorithmic (8 N^2: frame in, height out).", ""]
lines += ["Bench line of the profiled command:", "", "```json", json.dumps(pb), "```", "",
          "Unprofiled run of the same command on the same box:", "", "```json", bench, "```", ""]
open(dst, "w").write("\n".join(lines))
print("\n".join(lines))
