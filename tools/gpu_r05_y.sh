#!/bin/bash
# Round 5: the pointer-table encode (separately allocated blocks, the layout the
# JNI drop-in's encodeData hands over) under other write-window periods / widths
# with the three-slot ring, interleaved in one process (tools/kbench.py --tables),
# at k = 128 and k = 32; twice at k = 128.
# Run: gpurun -- 'bash tools/gpu_r05_y.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05y}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
L=ecwide_amd/libecwide.so
for i in 1 2; do
  timeout -k 10 400 python -u tools/kbench.py --tables --rounds 5 $L $L@11,32 $L@10,64 $L@12,64 $L@11,128 > $O/tables_k128_$i.log 2>&1 || { tail -20 $O/tables_k128_$i.log; exit 1; }
  tail -6 $O/tables_k128_$i.log
done
timeout -k 10 400 python -u tools/kbench.py --tables --k 32 --r 11 --m 3 --mib 64 --stripes 8 --rounds 5 $L $L@10,32 $L@11,64 $L@9,64 > $O/tables_k32.log 2>&1 || { tail -20 $O/tables_k32.log; exit 1; }
tail -5 $O/tables_k32.log
