#!/bin/bash
# Round 4: the N > 1 bench path on this one GPU (ranks share it): the self-
# launched --gpus 2 run, and the driver's own torchrun command at N = 2.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --gpus 2 --cpu-seconds 4 > gpurun_out/r04_bench_2rank_1gpu.log 2>&1
tail -1 gpurun_out/r04_bench_2rank_1gpu.log | cut -c1-300
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 2 --cpu-seconds 4 > gpurun_out/r04_bench_torchrun_n2_1gpu.log 2>&1
tail -1 gpurun_out/r04_bench_torchrun_n2_1gpu.log | cut -c1-300
