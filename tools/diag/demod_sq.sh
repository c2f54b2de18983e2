# SQ counters of the demod / fused kernels of the c2 bench: one
# rocprofv3 --pmc pass per counter group (at most 8 SQ counters each, --kernel-trace only),
# summarised per frame by tools/diag/sq_md.py.
# Usage (repo root on the box): TAG=r06x bash tools/diag/demod_sq.sh [bench args]
set -o pipefail
out=gpurun_out/${TAG:-r06sq}
mkdir -p $out
export TMPDIR=/tmp
args=${*:---steps 2 --warmup 1 --no-cpu-baseline --no-real-frames}
re='band_phase_res|k_phase_rows|demod_rows|demod_cols|demod_phase|int_cols|int_c2r'
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LEVEL_WAVES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$re" -f csv -d $out/sq$i -o run -- python3 bench.py $args > $out/sq$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/sq$i.log; exit 1; }
  echo "pass $i done"
done
python3 tools/diag/sq_md.py $out > $out/sq.md && cat $out/sq.md
