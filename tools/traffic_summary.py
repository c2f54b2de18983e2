"""HBM bytes per launch from the PMC passes of tools/traffic.sh.

    python tools/traffic_summary.py gpurun_out/<tag> [--frame 1024]

Calibration (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half the bytes of a wide
streaming read; other widths uncalibrated): the membench copies move a known
512 MiB per launch at 4, 8 and 16 B per lane, which gives the FETCH_SIZE and
WRITE_SIZE scale of each width on this pool.  The engine's kernels are scaled
with the factor of the width their dominant stream uses (measured, printed).
Writes profiles/traffic_<frame>.json for bench.py (roofline.traffic at that frame
size) and prints a per-kernel table.
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the demod launch group of bench.py's roofline pass: the band kernel (k_band_phase_res;
# at 4096 its 512-bin form since round 6; k_demod_phase before, and where no band fits)
DEMOD = ("k_demod_rows", "k_demod_cols", "k_band_phase", "k_demod_phase")
# the heights-only headline path (fused band transform + unwrap + row FFT)
HEADLINE = ("k_demod_rows", "k_demod_cols", "k_phase_rows", "k_colk", "k_seam_check", "k_int_cols", "k_int_c2r")
CHAIN = DEMOD + ("k_phase_rows", "k_seam_check", "k_colk", "k_int_rows2", "k_int_cols", "k_int_c2r")


def per_dispatch(path):
    rows = defaultdict(dict)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            d = rows[(f, r["Dispatch_Id"])]
            d["name"] = r["Kernel_Name"]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return list(rows.values())


def short(n):
    for k in CHAIN + ("copyk<float>", "copyk<HIP_vector_type<float, 2u> >", "copyk<HIP_vector_type<float, 4u> >", "strided"):
        if k in n:
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--frame", type=int, default=None, help="frame size (default: from the bench line)")
    ap.add_argument("--chunk", type=int, default=None, help="frames per launch (kbench runs: tools/traffic_kb.sh)")
    ap.add_argument("--out", default=None,
                    help="where to write the summary (default profiles/traffic_<frame>.json, which bench.py reads)")
    a = ap.parse_args()
    known = 512 << 20
    cal = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for d in per_dispatch(os.path.join(a.dir, "cal_" + c)):
            k = short(d["name"])
            if k:
                cal.setdefault(k, {})[c] = known / (d[c] * 1024.0)  # true bytes per counted byte
    print("calibration (true bytes / counter bytes):", json.dumps(cal, indent=1))
    fetch_f = cal.get("copyk<float>", {}).get("FETCH_SIZE", 2.0)   # 4 B per lane streams
    fetch_f8 = cal.get("copyk<HIP_vector_type<float, 2u> >", {}).get("FETCH_SIZE", 2.0)
    write_f = cal.get("copyk<float>", {}).get("WRITE_SIZE", 1.0)
    # Per kernel, the full-chunk launches of the roofline pass: the largest dispatches.
    # (bench.py also launches these kernels on the 1-frame reference and, on the
    # headline path, on half chunks; averaging over every dispatch, as an earlier
    # version did, understated the band kernel's phase stream by a third.)
    vals = defaultdict(lambda: defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for d in per_dispatch(os.path.join(a.dir, c)):
            k = short(d["name"])
            if k in CHAIN:
                vals[k][c].append(d[c] * 1024.0)
    for k in vals:
        for c in vals[k]:
            top = max(vals[k][c])
            vals[k][c] = [v for v in vals[k][c] if v >= 0.9 * top]
    # demod_rows / band_phase stream 4-B lanes (frame, theta, phases); demod_cols 8-B tiles
    factor = {"k_demod_rows": fetch_f, "k_band_phase": fetch_f, "k_demod_phase": fetch_f, "k_demod_cols": fetch_f8}
    table = {}
    for k in CHAIN:
        if k not in vals:
            continue
        fr = statistics.mean(vals[k]["FETCH_SIZE"]) * factor.get(k, fetch_f8) if vals[k]["FETCH_SIZE"] else 0.0
        wr = statistics.mean(vals[k]["WRITE_SIZE"]) * write_f if vals[k]["WRITE_SIZE"] else 0.0
        table[k] = {"read_bytes_per_launch": fr, "write_bytes_per_launch": wr}
    group = sum(table[k]["read_bytes_per_launch"] + table[k]["write_bytes_per_launch"] for k in DEMOD if k in table)
    # chunk size: frames per launch from the bench log line
    chunk = a.chunk
    streams = 1
    for line in open(os.path.join(a.dir, "FETCH_SIZE.log")):
        if line.startswith("{"):
            b = json.loads(line)
            if chunk is None:
                chunk = int(round(b["roofline"]["frames_per_launch"]))
            if a.frame is None:
                a.frame = int(b["config"]["frame"])
            streams = int(b["config"].get("streams_per_chunk", 1))
    # frames per kept launch: the largest launches of every kernel are whole chunks (the
    # roofline pass for the demod kernels; bench.py's stage-timed headline pass runs each
    # chunk on one stream, so its headline kernels too: k_int_c2r writes exactly
    # chunk x 4 N^2 bytes there)
    del streams
    for k, t in table.items():
        fpl = chunk
        t["frames_per_launch"] = fpl
        t["bytes_per_frame"] = (t["read_bytes_per_launch"] + t["write_bytes_per_launch"]) / fpl if fpl else None
    headline = {k: table[k]["bytes_per_frame"] for k in HEADLINE if k in table}
    res = {"frame": a.frame, "chunk": chunk, "demod_group_bytes_per_launch": int(group),
           "demod_group_bytes_per_frame": int(group / chunk) if chunk else None,
           "algorithmic_bytes_per_frame": 12 * a.frame * a.frame,
           "headline_bytes_per_frame": int(sum(headline.values())) if len(headline) == len(HEADLINE) else None,
           "headline_kernels": headline,
           "headline_algorithmic_bytes_per_frame": 8 * a.frame * a.frame,
           "per_kernel": table, "calibration": cal,
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes ({os.path.basename(a.dir)}: "
                     f"{'tools/kbench' if a.chunk else 'bench.py'}, largest launches per kernel); "
                     "FETCH scaled by the membench 4/8-B-lane calibration, WRITE by the 4-B-lane one"}
    print(json.dumps(res, indent=1))
    if a.out is None:
        a.out = os.path.join(ROOT, "profiles", f"traffic_{a.frame}.json")
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
