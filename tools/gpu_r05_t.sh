#!/bin/bash
# Round 5: the write window on the 5-8-row and 9-16-row asm tiles (off in the
# product since round 2: -1.2 % at 2^11 on the 5-8-row tile), periods 2^10..2^12,
# block slab, one process per shape (tools/kbench.py).
# Run: gpurun -- 'bash tools/gpu_r05_t.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05t}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
L=ecwide_amd/libecwide.so
for shape in "128 6 27 64" "128 8 27 64" "32 6 8 16" "128 12 27 64" "32 12 8 16"; do
  set -- $shape
  timeout -k 10 400 python -u tools/kbench.py --k $1 --m $2 --r $3 --mib $4 --stripes 4 --rounds 5 --check $L@off $L@10,64 $L@11,64 $L@12,64 $L@11,32 > $O/kbench_k$1_m$2.log 2>&1 || { tail -20 $O/kbench_k$1_m$2.log; exit 1; }
  tail -6 $O/kbench_k$1_m$2.log
done
