#!/bin/bash
# Round 5, second check: the tiled slab's repair with its new default (K = 2 +
# write window on 8 KiB units) -- the GPU suite, the placement study again with
# "auto" = the new default, the counters of every (slab, schedule) with this
# run's own durations (rocprofv3 --pmc + --kernel-trace: the slowest slab per
# schedule), the default bench under the kernel tracer and plain, and the
# 2-rank rehearsal of the per-rank host-resident leg.
# Run: gpurun -- 'bash tools/gpu_r05_b.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05b}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
SCH="auto 1,0 2,0,11,64 4,0,11,64 2,1,11,64 2,0,10,32"
timeout -k 10 400 python -u tools/repair_placement.py --split-at 3 --scheds $SCH > $O/placement_3.log 2>&1 || { tail -20 $O/placement_3.log; exit 1; }
tail -14 $O/placement_3.log
Q="python3 $R/tools/repair_placement.py --pmc-reps 3 --scheds $SCH"
cd /tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum --kernel-trace --output-format csv -d $O/plat -o run -- $Q > $O/pmc_lat.log 2>&1 || echo "latency counter pass failed"
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum --kernel-trace --output-format csv -d $O/pwr -o run -- $Q > $O/pmc_wr.log 2>&1 || echo "write counter pass failed"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pfetch -o run -- $Q > $O/pmc_fetch.log 2>&1 || echo "fetch pass failed"
cd $R
for d in plat pwr pfetch; do
  c=$(find $O/$d -name '*counter_collection.csv' | head -1)
  k=$(find $O/$d -name '*kernel_trace.csv' | head -1)
  [ -n "$c" ] && python tools/repair_placement.py --pmc-reps 3 --scheds $SCH --summarize $c $k > $O/pmc_${d}_summary.txt 2>&1
  rm -f $(find $O/$d -name '*.csv' ! -name '*kernel_stats.csv') 2>/dev/null
done
tail -30 $O/pmc_plat_summary.txt
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --cpu-seconds 0 > $O/bench_traced.log 2> $O/trace.log || exit $?
tail -1 $O/bench_traced.log | cut -c1-300
cd $R
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
timeout -k 10 600 python bench.py --gpus 2 --steps 10 --configs4-steps 2 --shape-steps 2 --other-layout-steps 0 > $O/bench_2rank.log 2>&1 || exit $?
tail -1 $O/bench_2rank.log | cut -c1-300
