#!/bin/bash
# Round 5: the encode's placement tail. Five tiled slabs + one split slab side by
# side (tools/repair_placement.py --enc-scheds): every slab's encode under each
# write-window / tile-order setting, judged by the worst tiled slab, in two
# processes with different allocation orders.
# Run: gpurun -- 'bash tools/gpu_r05_c.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05c}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
ENC="auto on 10,32 12,128 11,128 auto+r on+r"
for i in 1 2; do
  timeout -k 10 400 python -u tools/repair_placement.py --split-at $((i * 2)) --scheds auto 1,0 --enc-scheds $ENC > $O/enc_placement_$i.log 2>&1 || { tail -20 $O/enc_placement_$i.log; exit 1; }
  tail -12 $O/enc_placement_$i.log
done
