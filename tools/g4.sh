set -o pipefail
export TMPDIR=/tmp
for e in 1 2 3 4; do echo "== exp $e"; timeout -k 10 60 trapped-modes-ltg_amd/tools/bin/kbench_e$e 1024 8 20 | grep band || exit 1; done
mkdir -p gpurun_out/pmc2
kb=trapped-modes-ltg_amd/tools/kbench
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d gpurun_out/pmc2/p$i -o run -- $kb 1024 8 3 > gpurun_out/pmc2/p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -3 gpurun_out/pmc2/p$i.log; }
done
