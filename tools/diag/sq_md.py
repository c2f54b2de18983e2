"""Per-frame SQ counter summary of tools/diag/demod_sq.sh's passes (rocprofv3 --pmc CSVs
sq*/run_counter_collection.csv).

    python tools/diag/sq_md.py gpurun_out/<tag>

Per kernel, over its launches of the largest grid: mean duration, counters per launch and
per frame (frames per launch from the bench: 256 for the roofline pass's demod group, 128
for the headline's two concurrent halves), and the issue fractions
ACTIVE_INST_VALU / WAVE_CYCLES, WAIT_INST_ANY / WAVE_CYCLES, LDS_BANK_CONFLICT / LDS_IDX_ACTIVE.
"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def short(n):
    n = n[5:] if n.startswith("void ") else n
    p = n.find("(")
    return n[:p] if p > 0 else n


FPL = None  # frames per launch of the roofline pass (the chunk), from the command line


def frames_of(name, grid_rank):
    # k_band_phase_res / k_demod_phase only run in the roofline pass (FPL frames per launch,
    # 256 at 1024^2); the other kernels' largest launches: FPL in the roofline pass, FPL / 2
    # in the headline's two halves (1024^2: 256 / 128)
    fpl = FPL or 256
    if "band_phase_res" in name or "demod_phase" in name:
        return fpl
    if "k_phase_rows" in name or "int_c" in name:
        return fpl // 2 if fpl == 256 else fpl
    return fpl if grid_rank == 0 else fpl // 2


def main(d):
    per = defaultdict(lambda: defaultdict(list))  # (kernel, grid) -> counter -> [per launch]
    for f in sorted(glob.glob(os.path.join(d, "sq*", "*counter_collection.csv"))):
        disp = defaultdict(lambda: defaultdict(float))
        meta = {}
        for r in csv.DictReader(open(f)):
            k = r["Dispatch_Id"]
            meta[k] = (short(r["Kernel_Name"]), int(r["Grid_Size"]))
            disp[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k]["_dur_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, cs in disp.items():
            for c, v in cs.items():
                per[meta[k]][c].append(v)
    by_kernel = defaultdict(list)
    for (name, grid) in per:
        by_kernel[name].append(grid)
    print("# SQ counters per frame (rocprofv3 --pmc, tools/diag/demod_sq.sh)\n")
    for name in sorted(by_kernel):
        grids = sorted(by_kernel[name], reverse=True)
        for rank, grid in enumerate(grids[:2]):
            cs = {c: statistics.mean(v) for c, v in per[(name, grid)].items()}
            nl = max(len(v) for v in per[(name, grid)].values())
            if nl < 2 and rank > 0:
                continue
            fr = frames_of(name, rank)
            wc = cs.get("SQ_WAVE_CYCLES", 0) or 1
            print(f"## `{name}` grid {grid} ({nl} launches x passes, {fr} frames per launch, {cs['_dur_us']:.1f} us per launch)\n")
            print("| counter | per launch | per frame |")
            print("|---|---|---|")
            for c in sorted(cs):
                if c.startswith("_"):
                    continue
                print(f"| {c} | {cs[c]:.4g} | {cs[c] / fr:.4g} |")
            print()
            act = cs.get("SQ_ACTIVE_INST_VALU")
            if act is not None:
                print(f"ACTIVE_INST_VALU / WAVE_CYCLES = {act / wc:.3f}; "
                      f"WAIT_INST_ANY / WAVE_CYCLES = {cs.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}; "
                      f"LDS_BANK_CONFLICT / LDS_IDX_ACTIVE = "
                      f"{cs.get('SQ_LDS_BANK_CONFLICT', 0) / max(cs.get('SQ_LDS_IDX_ACTIVE', 1), 1):.3f}\n")


if __name__ == "__main__":
    if len(sys.argv) > 2:
        FPL = int(sys.argv[2])
    main(sys.argv[1])
