"""Per-kernel summary of a rocprofv3 kernel trace (rocpd SQLite db or *_kernel_trace.csv).

    python tools/prof_summary.py <run_results.db | kernel_trace.csv> [--frames-per-launch N] [--out file.md]

Prints, per kernel: launches, average / min / max duration (us) and total ms,
sorted by total time; with --frames-per-launch also us per frame.  Used to turn
the raw trace from tools/gpu_check.sh into the committed profiles/*.md.
"""
import argparse
import csv
import sqlite3
import statistics
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(list)
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for name, dur in db.execute("select name, duration from kernels"):
            d[name].append(dur / 1e3)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                d[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return d


def short(name):
    n = name.replace("HIP_vector_type<float, 2u>", "float2")
    if n.startswith("void "):
        n = n[5:]
    p = n.find("(")
    return n[:p] if p > 0 else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frames-per-launch", type=float, default=0)
    ap.add_argument("--filter", default="fcdk::")
    ap.add_argument("--out")
    a = ap.parse_args()
    d = load(a.trace)
    rows = []
    for k, v in d.items():
        if a.filter and a.filter not in k:
            continue
        rows.append((sum(v), k, v))
    rows.sort(reverse=True)
    lines = ["| kernel | launches | avg us | min us | max us | total ms |" + (" us/frame |" if a.frames_per_launch else ""),
             "|---|---|---|---|---|---|" + ("---|" if a.frames_per_launch else "")]
    for tot, k, v in rows:
        line = f"| `{short(k)}` | {len(v)} | {statistics.mean(v):.2f} | {min(v):.2f} | {max(v):.2f} | {tot / 1e3:.3f} |"
        if a.frames_per_launch:
            line += f" {statistics.mean(v) / a.frames_per_launch:.3f} |"
        lines.append(line)
    txt = "\n".join(lines) + "\n"
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)
    sys.stdout.write(txt)


if __name__ == "__main__":
    main()
