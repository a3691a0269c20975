#!/bin/bash
# Round 4: does the encode's shallow in-flight depth (2 loads per wave) make it
# sensitive to block alignment the way the XOR was? The XOR kernel as a proxy:
# 32 sources, 2 / 4 / 8 loads in flight per wave (-DECW_XOR_WINDOW), K = 1 vs 4,
# over separately allocated blocks, stride-B and stride-B+4K carves, split slab.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for W in w2 w4; do
  timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall_$W.so --stripes 4 --rounds 3 --r 32 \
    --placements sep,carved0,carved4k,split --scheds 1,0 4,0 > gpurun_out/r04_proxy_$W.log 2>&1
done
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 --r 32 \
  --placements sep,carved0,carved4k,split --scheds 1,0 4,0 > gpurun_out/r04_proxy_w8.log 2>&1
