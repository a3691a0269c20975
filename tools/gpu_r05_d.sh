#!/bin/bash
# Round 5: the tiled repair's window parameters at K = 2 (period / width), by
# the worst of five side-by-side tiled slabs, two processes.
# Run: gpurun -- 'bash tools/gpu_r05_d.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05d}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
SCH="auto 1,0 2,0,11,32 2,0,11,128 2,0,12,64 2,0,12,128 2,0,12,256 2,0,13,256 2,1,12,128"
for i in 1 2; do
  timeout -k 10 400 python -u tools/repair_placement.py --split-at $((i * 2 + 1)) --rounds 5 --scheds $SCH > $O/win_placement_$i.log 2>&1 || { tail -20 $O/win_placement_$i.log; exit 1; }
  tail -14 $O/win_placement_$i.log
done
