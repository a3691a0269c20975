#!/bin/bash
# Round 4: the product's XOR schedule choice (skew K=4 for pointer sources)
# against overrides, the encode's write window per layout, and the default
# bench line. Run: gpurun -- 'bash tools/gpu_r04_b.sh'
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/repair_ab.py --stripes 4 --encode --enc-windows auto off on \
  --scheds auto 1,0 4,0 4,0,11,64 > gpurun_out/r04b_repair_ab_1.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --stripes 4 --encode --enc-windows auto off on \
  --scheds auto 1,0 4,0 4,0,11,64 --placements sep,carved4k,carved0,split,tiled > gpurun_out/r04b_repair_ab_2.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r04b_bench_default.log 2>&1
