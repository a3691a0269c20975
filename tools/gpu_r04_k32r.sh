#!/bin/bash
# Round 4: tiled-slab repair at the k = 32 shapes with the 16 KiB pieces: one
# workgroup per 4 KiB tile (K = 1) against K = 2 / 4 column tiles per workgroup
# (a 16 KiB unit is one whole group of 4), with and without the write window.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
S="1,0 2,0 4,0 4,0,11,64 4,1"
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 32 --rounds 4 --k 32 --m 2 \
  --r 8 --mib 16 --chunk 16384 --placements tiled --scheds $S > gpurun_out/r04_k32r_cfg1.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 8 --rounds 4 --k 32 --m 3 \
  --r 11 --mib 64 --chunk 16384 --placements tiled --scheds $S > gpurun_out/r04_k32r_cfg0.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib build/variants/skewall.so --stripes 8 --rounds 4 \
  --chunk 8192 --placements tiled --scheds 1,0 2,0 2,0,11,64 > gpurun_out/r04_k128r_tiled.log 2>&1
