#!/bin/bash
# Round 4: K = 8 with the write window against the default K = 4 + window, on
# separate allocations, the stride-B carve and the split slab (n = 27 and 9).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 \
  --placements sep,carved0,split --scheds 4,0,11,64 8,0,11,64 2,0,11,64 8,0,12,64 > gpurun_out/r04_k8_r27.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 --r 9 \
  --placements sep,split --scheds 4,0,11,64 8,0,11,64 > gpurun_out/r04_k8_r9.log 2>&1
