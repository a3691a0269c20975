#!/bin/bash
# Round 5: the 5-8-row asm tile with a three-slot ring (build/variants/nw2r3.so =
# -DECW_ASM_RING3_NW2=1) against the product, interleaved in one process per shape
# (tools/kbench.py --check: every parity block of every stripe equal), small-k
# parity of both builds first.
# Build first: python tools/variants.py nw2r3=-DECW_ASM_RING3_NW2=1
# Run: gpurun -- 'bash tools/gpu_r05_u.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05u}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
V=${VARIANT:-build/variants/nw2r3.so}
L=ecwide_amd/libecwide.so
for k in 3 4 5 6 7 9 31; do
  for mode in "--code C --r 2" "--code R" "--code C --r 1 --literal" "--code C --r 1"; do
    timeout -k 10 120 python -u tools/kbench.py --k $k --m 6 --mib 1 --stripes 4 --rounds 1 --iters 1 --check $mode $L $V >> $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
  done
done
if grep -q "parity differs" $O/check.log; then grep "parity differs" $O/check.log | head; exit 1; fi
echo "small-k parity: both builds equal ($(grep -c 'encode' $O/check.log) lines)"
for shape in "128 6 27 64" "128 8 27 64" "32 6 8 16" "32 5 8 16"; do
  set -- $shape
  timeout -k 10 400 python -u tools/kbench.py --k $1 --m $2 --r $3 --mib $4 --stripes 4 --rounds 6 --check $L $V > $O/kbench_k$1_m$2.log 2>&1 || { tail -20 $O/kbench_k$1_m$2.log; exit 1; }
  tail -3 $O/kbench_k$1_m$2.log
done
timeout -k 10 400 python -u tools/kbench.py --k 128 --m 6 --r 27 --mib 64 --stripes 4 --rounds 6 --tables $L $V > $O/kbench_tables_k128_m6.log 2>&1 || { tail -20 $O/kbench_tables_k128_m6.log; exit 1; }
tail -3 $O/kbench_tables_k128_m6.log
