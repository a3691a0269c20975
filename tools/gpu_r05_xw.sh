#!/bin/bash
# Round 5: loads in flight per wave of the straight-line XOR kernel
# (ECW_XOR_WINDOW: 8 in the product; 4 and 16 as builds) at the k = 32 shapes'
# source counts (r = 8, 11) and at r = 27, block slab, one process per shape.
# Build first: python tools/variants.py xw16=-DECW_XOR_WINDOW=16 xw4=-DECW_XOR_WINDOW=4
# Run: gpurun -- 'bash tools/gpu_r05_xw.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05xw}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
L=ecwide_amd/libecwide.so
for shape in "32 2 8 16 32" "32 3 11 64 8" "128 3 27 64 4"; do
  set -- $shape
  timeout -k 10 400 python -u tools/kbench.py --k $1 --m $2 --r $3 --mib $4 --stripes $5 --rounds 6 $L build/variants/xw4.so build/variants/xw16.so > $O/k$1_r$3.log 2>&1 || { tail -20 $O/k$1_r$3.log; exit 1; }
  tail -4 $O/k$1_r$3.log
done
