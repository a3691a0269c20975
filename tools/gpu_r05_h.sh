#!/bin/bash
# Round 5: the <= 4-row asm tile with a three-slot ring (build/variants/ring3.so =
# -DECW_ASM_RING=3) against the product build: parity of both builds at small k
# (every tail of the ring) and in every local mode, then the encode of five tiled
# slabs + one split slab through both builds in the same rounds, judged by the
# worst tiled slab, in two processes.
# Build first: python tools/variants.py ring3=-DECW_ASM_RING=3
# Run: gpurun -- 'bash tools/gpu_r05_h.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05h}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
V=${VARIANT:-build/variants/ring3.so}
for k in 3 4 5 6 7 8 9 31 128; do
  for mode in "--code C" "--code R" "--code C --literal"; do
    timeout -k 10 120 python -u tools/kbench.py --k $k --m 3 --r 4 --mib 1 --stripes 4 --rounds 1 --iters 1 --check $mode ecwide_amd/libecwide.so $V >> $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
  done
done
if grep -q "parity differs" $O/check.log; then grep "parity differs" $O/check.log | head; exit 1; fi
echo "small-k parity: both builds equal ($(grep -c 'encode' $O/check.log) lines)"
for i in 1 2; do
  timeout -k 10 500 python -u tools/repair_placement.py --split-at $((i * 2)) --scheds auto --enc-scheds auto --enc-libs $V > $O/placement_$i.log 2>&1 || { tail -20 $O/placement_$i.log; exit 1; }
  tail -12 $O/placement_$i.log
done
