#!/bin/bash
# Round 5: the 9-16-row asm tile with a three-slot ring (build/variants/nw4r3.so =
# -DECW_ASM_RING3_NW4=1) against the product; the product's 5-8-row tile (three
# slots since r05u) against -DECW_ASM_RING3_NW2=0 once more. Small-k parity of
# the builds first, then interleaved timings (tools/kbench.py --check).
# Build first: python tools/variants.py nw4r3=-DECW_ASM_RING3_NW4=1 nw2off=-DECW_ASM_RING3_NW2=0
# Run: gpurun -- 'bash tools/gpu_r05_v.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05v}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
V=build/variants/nw4r3.so
W=build/variants/nw2off.so
L=ecwide_amd/libecwide.so
for k in 3 4 5 6 7 9 31; do
  for mode in "--code C --r 2" "--code R" "--code C --r 1 --literal" "--code C --r 1"; do
    timeout -k 10 120 python -u tools/kbench.py --k $k --m 12 --mib 1 --stripes 4 --rounds 1 --iters 1 --check $mode $L $V >> $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
    timeout -k 10 120 python -u tools/kbench.py --k $k --m 6 --mib 1 --stripes 4 --rounds 1 --iters 1 --check $mode $L $W >> $O/check.log 2>&1 || { tail -20 $O/check.log; exit 1; }
  done
done
if grep -q "parity differs" $O/check.log; then grep "parity differs" $O/check.log | head; exit 1; fi
echo "small-k parity: builds equal ($(grep -c 'encode' $O/check.log) lines)"
for shape in "128 12 27 64" "128 16 27 64" "32 12 8 16" "64 9 16 32"; do
  set -- $shape
  timeout -k 10 400 python -u tools/kbench.py --k $1 --m $2 --r $3 --mib $4 --stripes 4 --rounds 6 --check $L $V > $O/kbench_k$1_m$2.log 2>&1 || { tail -20 $O/kbench_k$1_m$2.log; exit 1; }
  tail -3 $O/kbench_k$1_m$2.log
done
timeout -k 10 400 python -u tools/kbench.py --k 128 --m 12 --r 27 --mib 64 --stripes 4 --rounds 6 --tables $L $V > $O/kbench_tables_k128_m12.log 2>&1 || { tail -20 $O/kbench_tables_k128_m12.log; exit 1; }
tail -3 $O/kbench_tables_k128_m12.log
timeout -k 10 400 python -u tools/kbench.py --k 128 --m 8 --r 27 --mib 64 --stripes 4 --rounds 6 --check $L $W > $O/kbench_nw2_k128_m8.log 2>&1 || { tail -20 $O/kbench_nw2_k128_m8.log; exit 1; }
tail -3 $O/kbench_nw2_k128_m8.log
