#!/bin/bash
# Round 4 check of a tree: smoke, the GPU suite, the default bench's main leg
# under the kernel tracer, FETCH_SIZE / WRITE_SIZE passes at the bench shape,
# the XOR-schedule counter evidence (tools/repair_pmc.py: kernel trace,
# FETCH_SIZE, TCC read-latency counters), then the full default bench line.
# Run: gpurun -- 'TAG=r04x bash tools/gpu_r04_final.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r04f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final_$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 > $O/bench_traced.log 2> $O/trace.log || exit $?
tail -1 $O/bench_traced.log | cut -c1-300
P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --no-verify"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_tiled -o run -- $P > $O/fetch_tiled.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_tiled -o run -- $P > $O/write_tiled.log 2>&1 || exit $?
# the XOR schedules on the pointer-leg placement and the split slab
Q="python3 $R/tools/repair_pmc.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rtrace -o run -- $Q > $O/repair_traced.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/rfetch -o run -- $Q > $O/repair_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/rwrite -o run -- $Q > $O/repair_write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum --output-format csv -d $O/rlat -o run -- $Q > $O/repair_lat.log 2>&1 || echo "latency counter pass failed"
timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum --output-format csv -d $O/rtlb1 -o run -- $Q > $O/repair_tlb1.log 2>&1 || echo "UTCL1 counter pass failed"
timeout -s KILL 300 rocprofv3 --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d $O/rtlb2 -o run -- $Q > $O/repair_tlb2.log 2>&1 || echo "UTCL2 counter pass failed"
cd $R
for d in rfetch rwrite rlat rtlb1 rtlb2; do
  f=$(find $O/$d -name '*counter_collection.csv' | head -1)
  [ -n "$f" ] && python tools/repair_pmc.py --summarize $f >> $O/repair_pmc_summary.txt 2>&1
done
cat $O/repair_pmc_summary.txt
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
find $O -name "*stats.csv" | head
echo done
