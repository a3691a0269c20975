#!/bin/bash
# Round 5: the k = 32 BASELINE shapes (configs[1] CL(32, 8, 2) 16 MiB x 32 stripes,
# configs[0] CL(32, 11, 3) 64 MiB x 8) through the same placement study: five tiled
# slabs (16 KiB pieces) + one split slab, the repair's XOR schedules and the
# encode's write window (with the three-slot ring), judged by the worst slab.
# Run: gpurun -- 'bash tools/gpu_r05_p.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05p}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --scheds auto 1,0 2,0,11,64 4,0,11,64 4,0 --enc-scheds auto 11,32 10,32 11,64 > $O/cfg1.log 2>&1 || { tail -20 $O/cfg1.log; exit 1; }
sed -n '/per schedule over/,$p' $O/cfg1.log
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 11 --m 3 --mib 64 --stripes 8 --scheds auto 1,0 2,0,11,64 4,0,11,64 4,0 --enc-scheds auto 11,32 10,32 11,64 > $O/cfg0.log 2>&1 || { tail -20 $O/cfg0.log; exit 1; }
sed -n '/per schedule over/,$p' $O/cfg0.log
