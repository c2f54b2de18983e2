"""PMC bytes of the real-frame (exact MST) pass per kernel: FETCH_SIZE / WRITE_SIZE passes
over tools/fixup_bench.py 96 (tools/diag/fixup_traffic.sh), scaled by the membench
calibration of the same run (FETCH x counter ratio at 4-B lanes, WRITE x its own), with
the kernel durations of the counter runs (serialised dispatches: the bytes are the figure
to read; the rate is against the unprofiled rocprof durations in r04au_fixup_kernel_stats).
Usage: python tools/diag/fixup_traffic_md.py gpurun_out/r04ay profiles/r04ay_fixup_traffic.md"""
import collections
import csv
import statistics
import sys

# unprofiled per-launch durations (us) of the same kernels, profiles/r04au_fixup_kernel_stats.md
R04AU_US = {"k_mst_tile0": 6539.7, "k_int_rows2<1024, 3>": 586.5, "k_cg_hook<true>": 240.0, "k_residues": 105.8,
            "k_cg_finalize": 325.4}


def load(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((int(r["Grid_Size"]), float(r["Counter_Value"])))
    return d


def main():
    src, dst = sys.argv[1], sys.argv[2]
    f, w = load(f"{src}/FETCH_SIZE/run_counter_collection.csv"), load(f"{src}/WRITE_SIZE/run_counter_collection.csv")
    cf, cw = load(f"{src}/cal_FETCH_SIZE/run_counter_collection.csv"), load(f"{src}/cal_WRITE_SIZE/run_counter_collection.csv")
    true_kb = 512 * 1024  # membench copies 512 MiB per launch
    ff = true_kb / statistics.mean(v for _, v in cf["copyk<float>"])
    fw = true_kb / statistics.mean(v for _, v in cw["copyk<float>"])
    lines = ["# r04ay — PMC bytes of the real-frame pass (exact MST unwrap)", "",
             "`rocprofv3 --kernel-trace --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` (separate passes) over "
             "`python3 tools/fixup_bench.py 96` (96 real 1024² frames = 192 maps per call, 5 calls), "
             f"largest grid of each kernel, mean per launch. Calibration from the same run's membench copies: "
             f"FETCH x{ff:.2f}, WRITE x{fw:.2f}. GB/s uses the unprofiled launch durations of "
             "`profiles/r04au_fixup_kernel_stats.md` where listed.", "",
             "| kernel | launches | read MB | write MB | us (r04au) | GB/s | of 8 TB/s |", "|---|---|---|---|---|---|---|"]
    rows = []
    for name, vals in f.items():
        if not name.startswith("fcdk::"):
            continue
        g = max(x[0] for x in vals)
        fv = [v for gg, v in vals if gg == g]
        wv = [v for gg, v in w.get(name, []) if gg == g]
        rd = statistics.mean(fv) * ff / 1024
        wr = (statistics.mean(wv) * fw / 1024) if wv else 0.0
        rows.append((rd + wr, name, len(fv), rd, wr))
    for tot, name, n, rd, wr in sorted(rows, reverse=True)[:14]:
        short = name.replace("fcdk::", "")
        us = next((v for k, v in R04AU_US.items() if short.startswith(k) or short == k), None)
        rate = f"{tot / us * 1e3:.0f}" if us else ""  # MB / us = TB/s
        frac = f"{tot / us / 8:.3f}" if us else ""
        lines.append(f"| `{short}` | {n} | {rd:.1f} | {wr:.1f} | {us if us else ''} | {rate} | {frac} |")
    open(dst, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
