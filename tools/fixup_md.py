"""Write profiles/<name>.md from a tools/r03_measure.sh run's `fixup` step: the
rocprofv3 --kernel-trace --stats summary of tools/fixup_bench.py (real camera frames with
residues through the exact MST pass) and the unprofiled bench line.

    python tools/fixup_md.py gpurun_out/<tag> profiles/<name>.md
"""
import csv
import json
import os
import sys

src, dst = sys.argv[1], sys.argv[2]
rows = [r for r in csv.DictReader(open(os.path.join(src, "fixprof", "run_kernel_stats.csv"))) if "fcdk::" in r["Name"]]
line = [l for l in open(os.path.join(src, "fixup.log")) if l.startswith("{")][-1]
b = json.loads(line)
tot = sum(float(r["TotalDurationNs"]) for r in rows)


def short(n):
    n = n.replace("HIP_vector_type<float, 2u>", "float2")
    n = n[5:] if n.startswith("void ") else n
    return n[:n.find("(")] if "(" in n else n


out = [f"# {os.path.basename(dst)[:-3]} — real camera frames with residues (exact MST unwrap), "
       "rocprofv3 --kernel-trace --stats", "",
       "Command: `rocprofv3 --kernel-trace --stats -f csv -- python3 tools/fixup_bench.py 96` (the three real "
       "10-bit frames of `tests/golden/real_df.npz`, 7..1611 residues per map, tiled to 96 frames, "
       "device-resident; 1 warm-up + 3 timed + 1 stage-timed pass = 5 calls). Engine kernels only. Source: "
       f"`{src}/fixprof/run_kernel_stats.csv`.", "",
       f"Unprofiled run of the same script (`{src}/fixup.log`): **{b['value']:.1f} frames/s** "
       f"({b['ms_per_frame']:.3f} ms/frame; first pass {b['first_pass_ms']} ms, exact fix-up pass "
       f"{b['fixup_ms']} ms for {b['frames']} frames per call).", "",
       "| kernel | calls | avg us | total ms | share |", "|---|---|---|---|---|"]
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"])
    out.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {t / 1e6:.2f} | "
               f"{100 * t / tot:.1f} % |")
open(dst, "w").write("\n".join(out) + "\n")
print("\n".join(out[:14]))
