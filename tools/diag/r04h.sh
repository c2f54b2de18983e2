set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "two_level or real_df or unwrap_reference or random_residues or residue_counts or census" > gpurun_out/r04h/tests.log 2>&1 && tail -3 gpurun_out/r04h/tests.log &&
bash tools/ab.sh r04h 3 'python tools/fixup_bench.py 96' c99:FCD_T0_ROUNDS=99 c1:FCD_T0_ROUNDS=1 c2:FCD_T0_ROUNDS=2 c3:FCD_T0_ROUNDS=3 c4:FCD_T0_ROUNDS=4
