#!/bin/bash
# Round 4: XOR write window parameters and fan-in (r = 27 / 9 / 4 sources) per
# layout, skew 1 vs 4; encode window per layout. Run: gpurun -- 'bash tools/gpu_r04_c.sh'
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
S="1,0 1,0,11,64 4,0 4,0,11,64 4,0,11,32 4,0,10,64 4,0,12,128"
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 \
  --placements tiled,split,blocks,sep,carved0 --scheds $S > gpurun_out/r04c_r27.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 --r 9 \
  --placements split,sep,carved0,tiled --scheds $S > gpurun_out/r04c_r9.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 --r 4 \
  --placements sep,split,carved0,tiled --scheds $S > gpurun_out/r04c_r4.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 4 --rounds 3 --k 32 --r 11 \
  --mib 64 --placements split,sep,tiled --encode --enc-windows auto off on --scheds 1,0 4,0 4,0,11,64 \
  > gpurun_out/r04c_k32.log 2>&1
