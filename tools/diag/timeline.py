"""Headline-step timeline from a rocprofv3 --kernel-trace CSV of `bench.py --steps K
--warmup W --no-cpu-baseline --no-real-frames` (GPU box: tools/diag/timeline.sh).

    python tools/diag/timeline.py run_kernel_trace.csv [--steps K]

The engine's headline launches form repeating groups (k_demod_rows ... k_int_c2r on two
queues); takes the K timed steps as the window from the first k_demod_rows of step W+1 to
the last k_int_c2r of the last timed step (the heights-only steps come before the profiled
passes), and reports: the window's wall time, the union of kernel intervals (GPU busy),
the sum of kernel durations (concurrency = sum / busy), per-kernel sums, and the idle gaps
longer than 5 us.
"""
import argparse
import csv
from collections import defaultdict


def short(n):
    n = n[5:] if n.startswith("void ") else n
    p = n.find("(")
    return n[:p] if p > 0 else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.csv)) if "fcdk::" in r["Kernel_Name"]]
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"])
                 for r in rows))
    # steps: each headline step launches k_demod_rows twice (two halves); skip warmup + the
    # reference setup launch (1 frame)
    dr = [i for i, k in enumerate(ks) if k[2].startswith("fcdk::k_demod_rows")]
    per_step = 2
    first = dr[1 + a.warmup * per_step]
    last_dr = dr[1 + (a.warmup + a.steps) * per_step - 1]
    # the window ends at the last c2r that starts before the next step's first demod_rows
    nxt = dr[1 + (a.warmup + a.steps) * per_step] if len(dr) > 1 + (a.warmup + a.steps) * per_step else len(ks)
    win = [k for k in ks[first:nxt]]
    t0 = win[0][0]
    t1 = max(k[1] for k in win)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, n, q in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                if s - cur_e > 5000:
                    gaps.append((s - cur_e, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = sum(e - s for s, e, n, q in win)
    per = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n, q in win:
        per[n] += (e - s) / 1e3
        cnt[n] += 1
    wall = (t1 - t0) / 1e3
    print(f"window {wall:.1f} us for {a.steps} steps ({wall / a.steps:.1f} us/step); busy {busy / 1e3:.1f} us "
          f"({busy / 1e3 / wall:.3f}); kernel-time sum {tot / 1e3:.1f} us (concurrency {tot / max(busy, 1):.2f})")
    for n, v in sorted(per.items(), key=lambda x: -x[1]):
        print(f"  {n:45s} {cnt[n]:4d} launches {v / a.steps:9.1f} us/step")
    print("gaps > 5 us:", len(gaps), "total", sum(g for g, _ in gaps) / 1e3, "us; first:",
          [(round(g / 1e3, 1), n) for g, n in gaps[:10]])


if __name__ == "__main__":
    main()
