#!/bin/bash
# PMC passes over the kernel micro-benchmark (one counter group per pass,
# --kernel-trace only, never combined with sys/runtime traces).
# Usage on the GPU box: bash tools/pmc.sh <tag> [N] [nb]
set -o pipefail
tag=${1:-pmc}; N=${2:-1024}; nb=${3:-8}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
kb=trapped-modes-ltg_amd/tools/kbench
timeout -k 10 120 $kb $N $nb 10 > $out/kbench.txt 2>&1 || { echo "kbench failed"; cat $out/kbench.txt; exit 1; }
cat $out/kbench.txt
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F32" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -f csv -d $out/p$i -o run -- $kb $N $nb 3 > $out/p$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -3 $out/p$i.log; }
done
