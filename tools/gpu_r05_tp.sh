#!/bin/bash
# Round 5: column tiles per workgroup of the <= 4-row asm tile under the write
# window (the product: 1; build/variants/tpb2.so: 2, a workgroup of 512 threads
# encodes a whole 8 KiB piece and shares one LDS copy of the tables), five tiled
# slabs + one split slab, through both builds in the same rounds; two processes.
# Build first: python tools/variants.py tpb2=-DECW_ASM_TPB1=2
# Run: gpurun -- 'bash tools/gpu_r05_tp.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05tp}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
for i in 1 2; do
  timeout -k 10 500 python -u tools/repair_placement.py --split-at $((i * 2)) --rounds 4 --scheds auto --enc-scheds auto --enc-libs build/variants/tpb2.so > $O/placement_$i.log 2>&1 || { tail -20 $O/placement_$i.log; exit 1; }
  sed -n '/encode GB\/s per slab/,$p' $O/placement_$i.log
done
