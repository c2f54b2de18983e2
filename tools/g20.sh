# rehearse the N>1 bench path: 2 ranks sharing the box's one GPU over gloo
set -o pipefail
mkdir -p gpurun_out/r01k
FCD_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --batch 64 --gather > gpurun_out/r01k/bench2.log 2>&1 || { tail -30 gpurun_out/r01k/bench2.log; exit 1; }
grep '^{' gpurun_out/r01k/bench2.log
