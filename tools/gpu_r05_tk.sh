#!/bin/bash
# Round 5: the HBM-filling batch's launch shape under the write window: one
# ticket-ordered launch (the product, >= 4 launch windows of tiles) against launch
# windows (build/variants/noticket.so = -DECW_TICKET_MIN_TILES=0), one tiled slab of
# 240 stripes x 8 MiB blocks (261 GB), both builds in the same rounds.
# Build first: python tools/variants.py noticket=-DECW_TICKET_MIN_TILES=0
# Run: gpurun -- 'bash tools/gpu_r05_tk.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05tk}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u tools/repair_placement.py --slabs 1 --split 0 --stripes 240 --mib 8 --rounds 4 --scheds auto --enc-scheds auto --enc-libs build/variants/noticket.so > $O/hbmfill.log 2>&1 || { tail -20 $O/hbmfill.log; exit 1; }
sed -n '/encode GB\/s per slab/,$p' $O/hbmfill.log
