#!/bin/bash
# Round 5: the encode's launch shape under the write window: the product (launch
# windows of 65,536 tiles) against builds that take the slab as one ticket-ordered
# launch (-DECW_TICKET_MIN_TILES=1) or one grid-strided launch
# (-DECW_COHORT_TILES=-1), on five tiled slabs + one split slab, two processes.
# Build first: python tools/variants.py ticket=-DECW_TICKET_MIN_TILES=1 onelaunch=-DECW_COHORT_TILES=-1
# Run: gpurun -- 'bash tools/gpu_r05_n.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05n}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u tools/repair_placement.py --split-at $((i * 2)) --scheds auto --enc-scheds auto --enc-libs build/variants/ticket.so build/variants/onelaunch.so > $O/placement_$i.log 2>&1 || { tail -20 $O/placement_$i.log; exit 1; }
  sed -n '/encode GB\/s per slab/,$p' $O/placement_$i.log
done
