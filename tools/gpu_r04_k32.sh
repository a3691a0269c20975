#!/bin/bash
# Round 4: tiled piece size at the k=32 BASELINE shapes (configs[1]: CL(32,8,2)
# 16 MiB x 32 stripes; the default scheme.ini shape CL(32,11,3) 64 MiB x 8), one
# allocation per process, variants interleaved (tools/layout_ab.py).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
V="tiled:4096:0,tiled:8192:0,tiled:16384:0,tiled:32768:0,tiled:65536:0,blocks:4096"
timeout -k 10 300 python -u tools/layout_ab.py --k 32 --m 2 --r 8 --mib 16 --stripes 32 --rounds 4 --variants $V \
  > gpurun_out/r04_k32_piece_cfg1.log 2>&1
timeout -k 10 300 python -u tools/layout_ab.py --k 32 --m 3 --r 11 --mib 64 --stripes 8 --rounds 4 --variants $V \
  > gpurun_out/r04_k32_piece_cfg0.log 2>&1
timeout -k 10 300 python -u tools/layout_ab.py --k 128 --m 3 --r 27 --mib 64 --stripes 8 --rounds 3 \
  --variants tiled:8192:0,tiled:16384:0,tiled:4096:0 > gpurun_out/r04_k128_piece.log 2>&1
timeout -k 10 400 python -u tools/cpu_baseline.py > gpurun_out/r04_cpu_baselines.log 2>&1
# tiled slab repair: K = 2 (both 4 KiB tiles of an 8 KiB unit in one workgroup), column-major order
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 8 --rounds 4 \
  --placements tiled --scheds 1,0 2,0 1,1 2,1 > gpurun_out/r04_tiled_repair_k2.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 32 --rounds 4 --k 32 --m 2 \
  --r 8 --mib 16 --placements tiled --scheds 1,0 2,0 1,1 2,1 > gpurun_out/r04_tiled_repair_k2_cfg1.log 2>&1
