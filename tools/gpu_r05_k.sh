#!/bin/bash
# Round 5: the tiled encode with the write window forced on, now that the window
# brings the three-slot ring with it (five tiled slabs + one split slab, worst
# tiled slab decides, two processes).
# Run: gpurun -- 'bash tools/gpu_r05_k.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05k}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u tools/repair_placement.py --split-at $((i * 2)) --scheds auto --enc-scheds auto on 11,128 12,128 10,32 > $O/placement_$i.log 2>&1 || { tail -20 $O/placement_$i.log; exit 1; }
  tail -9 $O/placement_$i.log
done
