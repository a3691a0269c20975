#!/bin/bash
# Round 5: the encode window from k = 32 on (2^10 ticks below k = 64): the window
# parity tests, then the block slab and pointer tables at k = 16 / 24 / 32 / 48
# with the window off / the library's choice / forced periods (tools/kbench.py,
# one process each), the k = 32 shapes' placement study (auto vs off), the bench.
# Run: gpurun -- 'bash tools/gpu_r05_r.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05r}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "window" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_window.log 2>&1 || { tail -40 $O/pytest_window.log; exit 1; }
tail -2 $O/pytest_window.log
L=ecwide_amd/libecwide.so
for k in 16 24 32 48; do
  timeout -k 10 300 python -u tools/kbench.py --k $k --m 3 --r 8 --mib 16 --stripes 16 --rounds 5 --check $L@off $L $L@10,64 $L@11,64 $L@9,64 > $O/kbench_k$k.log 2>&1 || { tail -20 $O/kbench_k$k.log; exit 1; }
  tail -6 $O/kbench_k$k.log
done
for k in 32 48; do
  timeout -k 10 300 python -u tools/kbench.py --k $k --m 3 --r 8 --mib 16 --stripes 16 --rounds 5 --tables $L@off $L $L@11,64 > $O/kbench_tables_k$k.log 2>&1 || { tail -20 $O/kbench_tables_k$k.log; exit 1; }
  tail -4 $O/kbench_tables_k$k.log
done
timeout -k 10 500 python -u tools/repair_placement.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --scheds auto --rounds 4 --enc-scheds auto off > $O/cfg1.log 2>&1 || { tail -20 $O/cfg1.log; exit 1; }
sed -n '/per encode schedule/,$p' $O/cfg1.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
