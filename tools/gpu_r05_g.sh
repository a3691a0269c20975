#!/bin/bash
# Round 5, check of the tree with the paired K = 4 repair default: smoke, the
# GPU suite, the placement study (auto = paired K = 4 + window) in one process,
# the default bench under the kernel tracer and plain, FETCH / WRITE passes of
# the bench's repair, and configs[3] (--hbm-fill) under the tracer; with
# TWO_RANK=1 also bench.py --gpus 2 with both ranks on the one GPU.
# Run: gpurun -- 'bash tools/gpu_r05_g.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05g}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u tools/repair_placement.py --split-at 1 --scheds auto 2,0,11,64 4,0,11,64 1,0 > $O/placement_g.log 2>&1 || { tail -20 $O/placement_g.log; exit 1; }
tail -9 $O/placement_g.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --cpu-seconds 0 > $O/bench_traced.log 2> $O/trace.log || exit $?
tail -1 $O/bench_traced.log | cut -c1-200
P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --no-verify"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $P > $O/write.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hftrace -o run -- python3 $R/bench.py --hbm-fill --steps 5 --warmup 1 --cpu-seconds 0 --host-iters 0 > $O/hbmfill_traced.log 2> $O/hftrace.log || exit $?
tail -1 $O/hbmfill_traced.log | cut -c1-200
cd $R
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
if [ -n "${TWO_RANK:-}" ]; then
  timeout -k 10 600 python bench.py --gpus 2 --steps 10 --configs4-steps 2 --shape-steps 2 --other-layout-steps 0 > $O/bench_2rank.log 2>&1 || exit $?
  tail -1 $O/bench_2rank.log | cut -c1-300
fi
