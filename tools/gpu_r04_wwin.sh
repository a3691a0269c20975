#!/bin/bash
# Round 4: the encode write window's period / width for pointer tables over
# separate allocations, now with the per-XCD tile order (and the split slab).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/repair_ab.py --stripes 4 --rounds 3 --encode \
  --enc-windows auto 11,32 11,128 10,32 10,64 12,64 12,128 --placements sep,split,tiled --scheds auto \
  > gpurun_out/r04_wwin_ptr.log 2>&1
