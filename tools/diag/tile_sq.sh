# SQ counters of the real-frame pass (one --pmc pass, SQ block only): LDS bank-conflict
# cycles against all LDS cycles, wave-parked vs issue-stalled vs issuing cycles
set -o pipefail
out=gpurun_out/${TAG:-r04bc}
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS --kernel-include-regex 'mst_tile0|cg_hook|int_rows2' -f csv -d $out/sq -o run -- python3 tools/fixup_bench.py 96 > $out/sq.log 2>&1 || { tail -5 $out/sq.log; exit 1; }
echo sq done
