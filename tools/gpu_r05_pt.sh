#!/bin/bash
# Round 5: two column tiles per workgroup (build/variants/tpb2.so =
# -DECW_ASM_TPB1=2: 8 KiB of a row per workgroup, half the address translations per
# byte) for the pointer-table encode over separately allocated blocks, the layout
# whose encode is translation-bound; k = 128 and k = 32, twice at k = 128.
# Build first: python tools/variants.py tpb2=-DECW_ASM_TPB1=2
# Run: gpurun -- 'bash tools/gpu_r05_pt.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05pt}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
L=ecwide_amd/libecwide.so
V=build/variants/tpb2.so
for i in 1 2; do
  timeout -k 10 400 python -u tools/kbench.py --tables --rounds 6 $L $V > $O/tables_k128_$i.log 2>&1 || { tail -20 $O/tables_k128_$i.log; exit 1; }
  tail -3 $O/tables_k128_$i.log
done
timeout -k 10 400 python -u tools/kbench.py --tables --k 32 --r 11 --m 3 --mib 64 --stripes 8 --rounds 6 $L $V > $O/tables_k32.log 2>&1 || { tail -20 $O/tables_k32.log; exit 1; }
tail -3 $O/tables_k32.log
timeout -k 10 400 python -u tools/kbench.py --rounds 6 --check $L $V > $O/blocks_k128.log 2>&1 || { tail -20 $O/blocks_k128.log; exit 1; }
tail -3 $O/blocks_k128.log
