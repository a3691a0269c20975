#!/bin/bash
# Round 5: the tiled encode's write-window period / width (with the three-slot
# ring it brings), judged by the worst of five tiled slabs, three processes with
# the split slab at different positions in the allocation order.
# Run: gpurun -- 'bash tools/gpu_r05_l.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05l}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
for i in 0 1 2; do
  timeout -k 10 500 python -u tools/repair_placement.py --split-at $((i * 2 + 1)) --scheds auto --enc-scheds off 10,32 11,64 10,64 9,16 11,32 > $O/placement_$i.log 2>&1 || { tail -20 $O/placement_$i.log; exit 1; }
  tail -9 $O/placement_$i.log
done
