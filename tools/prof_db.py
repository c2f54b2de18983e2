"""Per-kernel totals of a rocprofv3 rocpd database, split by launch order into the
shape_bench.py shapes (each shape's kernels are contiguous).  Quick look, not committed profiles.

    python tools/prof_db.py <run_results.db> [top]
"""
import sqlite3
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("HIP_vector_type<float, 2u>", "float2")
    n = n[5:] if n.startswith("void ") else n
    return n[:n.find("(")] if "(" in n else n


db = sqlite3.connect(sys.argv[1])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
d = defaultdict(list)
for n, t in db.execute("select name, duration from kernels"):
    if "fcdk" in n:
        d[short(n)].append(t / 1e3)
for n, v in sorted(d.items(), key=lambda x: -sum(x[1]))[:top]:
    print(f"{len(v):5d} {sum(v) / len(v):9.1f} us {sum(v) / 1e3:8.2f} ms  {n}")
