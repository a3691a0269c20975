#!/bin/bash
# Round 5: the encode write window's period against the stripe width: at the
# k = 32 shapes (configs[1], configs[0]) a 2^10-tick period gains where 2^11 did
# not; sweep period / width there and at k = 128, five tiled slabs + one split
# slab each, worst slab decides.
# Run: gpurun -- 'bash tools/gpu_r05_q.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05q}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
P="--scheds auto --rounds 4"
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 $P --enc-scheds off 10,32 10,16 10,64 9,16 9,32 > $O/cfg1.log 2>&1 || { tail -20 $O/cfg1.log; exit 1; }
sed -n '/per encode schedule/,$p' $O/cfg1.log
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 11 --m 3 --mib 64 --stripes 8 $P --enc-scheds off 10,32 10,16 10,64 9,16 9,32 > $O/cfg0.log 2>&1 || { tail -20 $O/cfg0.log; exit 1; }
sed -n '/per encode schedule/,$p' $O/cfg0.log
timeout -k 10 500 python -u tools/repair_placement.py $P --enc-scheds off 11,32 10,32 10,16 11,16 > $O/k128.log 2>&1 || { tail -20 $O/k128.log; exit 1; }
sed -n '/per encode schedule/,$p' $O/k128.log
