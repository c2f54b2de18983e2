"""Summarise rocprofv3 --pmc CSV passes (tools/pmc.sh) per kernel.

    python tools/pmc_summary.py gpurun_out/<tag> [--frames-per-launch 8]

Per kernel: mean duration and the mean of every counter collected in the passes
p*/run_counter_collection.csv.  FETCH_SIZE / WRITE_SIZE are in KiB as rocprofv3
reports them; HBM bytes per launch = 2 * FETCH_SIZE * 1024 (gfx950 reports half
the bytes of wide streaming reads, MI355X_MICROARCH.md §HBM) + WRITE_SIZE * 1024.
"""
import argparse
import csv
import glob
import os
import statistics
from collections import defaultdict


def short(n):
    n = n.replace("HIP_vector_type<float, 2u>", "float2")
    n = n[5:] if n.startswith("void ") else n
    p = n.find("(")
    return n[:p] if p > 0 else n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--frames-per-launch", type=float, default=8)
    ap.add_argument("--filter", default="fcdk::")
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "*counter_collection.csv"))):
        per_dispatch = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            if a.filter not in r["Kernel_Name"]:
                continue
            d = r["Dispatch_Id"]
            names[d] = short(r["Kernel_Name"])
            per_dispatch[d][r["Counter_Name"]] += float(r["Counter_Value"])
            per_dispatch[d]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per_dispatch[d]["_vgpr"] = float(r["VGPR_Count"])
            per_dispatch[d]["_lds"] = float(r["LDS_Block_Size"])
            per_dispatch[d]["_grid"] = float(r["Grid_Size"])
            per_dispatch[d]["_wg"] = float(r["Workgroup_Size"])
        for d, cs in per_dispatch.items():
            for c, v in cs.items():
                vals[names[d]][c].append(v)
    fpl = a.frames_per_launch
    for k, cs in vals.items():
        m = {c: statistics.mean(v) for c, v in cs.items()}
        print(f"== {k}  (vgpr {m.get('_vgpr', 0):.0f}, lds {m.get('_lds', 0):.0f} B, grid {m.get('_grid', 0):.0f}, wg {m.get('_wg', 0):.0f})")
        line = []
        for c in sorted(m):
            if not c.startswith("_"):
                line.append(f"{c}={m[c]:.4g}")
        print("   " + "  ".join(line))
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            rd = 2 * m.get("FETCH_SIZE", 0) * 1024 / fpl / 1e6
            wr = m.get("WRITE_SIZE", 0) * 1024 / fpl / 1e6
            print(f"   HBM-side per frame: read {rd:.2f} MB (FETCH x2), write {wr:.2f} MB")
        if "SQ_INSTS_VALU" in m:
            print(f"   per frame: VALU wave-instr {m['SQ_INSTS_VALU'] / fpl / 1e6:.3f} M, LDS wave-instr "
                  f"{m.get('SQ_INSTS_LDS', 0) / fpl / 1e6:.3f} M, SALU {m.get('SQ_INSTS_SALU', 0) / fpl / 1e6:.3f} M")
        if "SQ_BUSY_CYCLES" in m and "SQ_ACTIVE_INST_VALU" in m:
            print(f"   ACTIVE_VALU/WAVE_CYCLES {m['SQ_ACTIVE_INST_VALU'] / max(m['SQ_WAVE_CYCLES'], 1):.3f}  "
                  f"ACTIVE_LDS/WAVE_CYCLES {m.get('SQ_ACTIVE_INST_LDS', 0) / max(m['SQ_WAVE_CYCLES'], 1):.3f}")
        if "SQ_LDS_IDX_ACTIVE" in m:
            print(f"   LDS bank conflict / idx active {m['SQ_LDS_BANK_CONFLICT'] / max(m['SQ_LDS_IDX_ACTIVE'], 1):.3f}, "
                  f"unaligned stall / idx active {m.get('SQ_LDS_UNALIGNED_STALL', 0) / max(m['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
        if "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
            wc = max(m["SQ_WAVE_CYCLES"], 1)
            print(f"   wave time: waitcnt/barrier {m['SQ_WAIT_ANY'] / wc:.2f}, issue-stall {m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}, "
                  f"active {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}; mean resident waves/CU "
                  f"{m.get('SQ_LEVEL_WAVES', 0) / max(m.get('SQ_BUSY_CYCLES', 1), 1) / 256 * 4 if m.get('SQ_LEVEL_WAVES') else 0:.1f}")
        if "SQ_THREAD_CYCLES_VALU" in m and "SQ_ACTIVE_INST_VALU" in m:
            print(f"   VALU lane utilisation {m['SQ_THREAD_CYCLES_VALU'] / max(64 * m['SQ_ACTIVE_INST_VALU'], 1):.2f}")
        if "_dur" in m and "SQ_ACTIVE_INST_VALU" in m:
            # ACTIVE_INST_VALU counts quad-cycles summed over waves; 1024 SIMDs
            print(f"   VALU busy per SIMD: {m['SQ_ACTIVE_INST_VALU'] * 4 / 1024 / (m['_dur'] * 1e-6 * 2.4e9):.2f} (at 2.4 GHz)")


if __name__ == "__main__":
    main()
