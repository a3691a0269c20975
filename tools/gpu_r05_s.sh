#!/bin/bash
# Round 5: the repair's XOR write-window period against the source count (r = 8
# and 11 at the k = 32 shapes, 27 at the bench's), and the k = 128 encode at
# 2^12; five tiled slabs + one split slab each, worst slab decides.
# Run: gpurun -- 'bash tools/gpu_r05_s.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05s}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
S="auto 4,0,10,64 4,0,10,32 4,0,9,32 4,0,9,16 4,0,12,64"
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --rounds 4 --scheds $S > $O/cfg1.log 2>&1 || { tail -20 $O/cfg1.log; exit 1; }
sed -n '/per schedule over/,$p' $O/cfg1.log
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 11 --m 3 --mib 64 --stripes 8 --rounds 4 --scheds $S > $O/cfg0.log 2>&1 || { tail -20 $O/cfg0.log; exit 1; }
sed -n '/per schedule over/,$p' $O/cfg0.log
timeout -k 10 500 python -u tools/repair_placement.py --rounds 4 --scheds auto 4,0,12,64 4,0,10,64 4,0,12,32 --enc-scheds auto 12,32 12,64 11,16 > $O/k128.log 2>&1 || { tail -20 $O/k128.log; exit 1; }
sed -n '/per schedule over/,$p' $O/k128.log
