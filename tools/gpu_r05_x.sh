#!/bin/bash
# Round 5: the tiled slab's piece size under the round-5 schedules (windowed
# encode with three ring slots, paired / whole-group K = 4 repair), all variants
# carved from ONE allocation and interleaved (tools/layout_ab.py), at the bench
# shape and at the k = 32 shapes; twice at k = 128 (two processes).
# Run: gpurun -- 'bash tools/gpu_r05_x.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
V="blocks:4096,tiled:4096:0,tiled:8192:0,tiled:16384:0,tiled:32768:0"
for i in 1 2; do
  timeout -k 10 400 python -u tools/layout_ab.py --rounds 4 --variants $V > $O/k128_$i.log 2>&1 || { tail -20 $O/k128_$i.log; exit 1; }
  tail -6 $O/k128_$i.log
done
timeout -k 10 400 python -u tools/layout_ab.py --k 32 --r 11 --m 3 --mib 64 --stripes 8 --rounds 4 --variants "blocks:4096,tiled:8192:0,tiled:16384:0,tiled:32768:0" > $O/cfg0.log 2>&1 || { tail -20 $O/cfg0.log; exit 1; }
tail -5 $O/cfg0.log
timeout -k 10 400 python -u tools/layout_ab.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --rounds 4 --variants "blocks:4096,tiled:8192:0,tiled:16384:0,tiled:32768:0" > $O/cfg1.log 2>&1 || { tail -20 $O/cfg1.log; exit 1; }
tail -5 $O/cfg1.log
