set -o pipefail
export AMD_SERIALIZE_KERNEL=3 HIP_LAUNCH_BLOCKING=1
timeout -k 10 300 python -m pytest tests -m gpu -x -q ${PYK:+-k "$PYK"} > gpurun_out/pytest_one.log 2>&1; rc=$?
grep -E "Error|error|passed|failed" gpurun_out/pytest_one.log | head -20
exit $rc
