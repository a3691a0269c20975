#!/bin/bash
# The maintained final-tree check (round 6 on). PART=a: smoke, the GPU suite,
# the default bench line, the N=2 path rehearsed on one GPU (both ranks share
# it) plain and with an injected failure in the host leg. PART=b: the
# profiles the line's roofline cites -- the main leg under the kernel tracer
# (-> profiles/<TAG>_bench_kernel_stats.csv), FETCH_SIZE / WRITE_SIZE passes
# (-> pmc_traffic*.json via tools/prof_summary.py), configs[3] traced -- and
# the N=2 hang rehearsal (a rank stops in a leg; the other's collective times
# out; rank 0 still prints). Each GPU step has its own limit; the script stops
# at the first failure. PART=c: the N>1 orchestration with 4 real GPU
# processes sharing the one GPU (16 MiB main-leg blocks so four ranks fit),
# plain, with a rank hanging in a leg and with a rank exiting mid-leg -- the
# line must come out every time -- and the new 2-rank GPU test.
# Run: gpurun -- 'TAG=r06a PART=a bash tools/gpu_final.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r06}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
if [ "${PART:-a}" = a ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 400 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
  tail -1 $O/bench_default.log | cut -c1-300
  timeout -k 10 400 python bench.py --gpus 2 --steps 10 --configs4-steps 2 --shape-steps 2 --other-layout-steps 0 > $O/bench_2rank.log 2>&1 || { tail -20 $O/bench_2rank.log; exit 1; }
  tail -1 $O/bench_2rank.log | cut -c1-300
  timeout -k 10 400 python bench.py --gpus 2 --steps 10 --configs4-steps 2 --shape-steps 2 --other-layout-steps 0 --inject-fail rank=1,leg=host > $O/bench_2rank_fail_host.log 2>&1 || { tail -20 $O/bench_2rank_fail_host.log; exit 1; }
  tail -1 $O/bench_2rank_fail_host.log | cut -c1-300
fi
if [ "${PART:-a}" = b ]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --cpu-seconds 0 > $O/bench_traced.log 2> $O/trace.log || exit $?
  tail -1 $O/bench_traced.log | cut -c1-200
  P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --no-verify"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hftrace -o run -- python3 $R/bench.py --hbm-fill --steps 5 --warmup 1 --cpu-seconds 0 --host-iters 0 > $O/hbmfill_traced.log 2> $O/hftrace.log || exit $?
  tail -1 $O/hbmfill_traced.log | cut -c1-200
  cd $R
  timeout -k 10 400 python bench.py --gpus 2 --steps 10 --configs4-steps 2 --shape-steps 2 --other-layout-steps 0 --inject-fail rank=1,leg=configs1,at=1,mode=hang --collective-timeout 20 --deadline-s 240 > $O/bench_2rank_hang.log 2>&1 || { tail -20 $O/bench_2rank_hang.log; exit 1; }
  tail -1 $O/bench_2rank_hang.log | cut -c1-300
fi
if [ "${PART:-a}" = c ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 280 --timeout-method thread -p no:cacheprovider > $O/pytest_multirank.log 2>&1 || { tail -40 $O/pytest_multirank.log; exit 1; }
  tail -2 $O/pytest_multirank.log
  Q="--block-mib 16 --steps 10 --configs4-steps 2 --shape-steps 2 --other-layout-steps 0"
  timeout -k 10 400 python bench.py --gpus 4 $Q > $O/bench_4rank.log 2>&1 || { tail -20 $O/bench_4rank.log; exit 1; }
  tail -1 $O/bench_4rank.log | cut -c1-300
  timeout -k 10 400 python bench.py --gpus 4 $Q --inject-fail rank=2,leg=configs0_shape,at=1,mode=hang --collective-timeout 30 > $O/bench_4rank_hang.log 2>&1 || { tail -20 $O/bench_4rank_hang.log; exit 1; }
  tail -1 $O/bench_4rank_hang.log | cut -c1-300
  timeout -k 10 400 python bench.py --gpus 4 $Q --inject-fail rank=3,leg=configs4,at=2,mode=exit > $O/bench_4rank_exit.log 2>&1; echo "exit-mode rc=$?"
  tail -1 $O/bench_4rank_exit.log | cut -c1-300
fi
