#!/bin/bash
# Round 5: workgroups per CU of the encode's launch windows under the write window
# (the product: 256, one tile per workgroup; 128 / 64 / 24: each workgroup takes
# several tiles grid-strided and stages its LDS tables once), five tiled slabs +
# one split slab, through the builds in the same rounds; two processes.
# Build first: python tools/variants.py g64=-DECW_GRID_PER_CU=64 g128=-DECW_GRID_PER_CU=128 g24=-DECW_GRID_PER_CU=24
# Run: gpurun -- 'bash tools/gpu_r05_z.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05z}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u tools/repair_placement.py --split-at $((i * 2)) --rounds 4 --scheds auto --enc-scheds auto --enc-libs build/variants/g128.so build/variants/g64.so build/variants/g24.so > $O/placement_$i.log 2>&1 || { tail -20 $O/placement_$i.log; exit 1; }
  sed -n '/encode GB\/s per slab/,$p' $O/placement_$i.log
done
