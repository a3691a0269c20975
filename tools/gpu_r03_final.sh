# Round 3, final tree: smoke, the GPU suite, the main leg of the default bench
# under the kernel tracer, FETCH_SIZE / WRITE_SIZE passes at the bench shape,
# then the full default bench line (what the driver runs).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r03f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/final_$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 --configs4-steps 0 --host-iters 0 > $O/bench_traced.log 2> $O/trace.log || exit $?
tail -1 $O/bench_traced.log | cut -c1-400
P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0 --configs4-steps 0 --host-iters 0 --no-verify"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_tiled -o run -- $P > $O/fetch_tiled.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_tiled -o run -- $P > $O/write_tiled.log 2>&1 || exit $?
cd $R
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-400
find $O -name "*stats.csv" | head

# the N = 2 path on this one GPU (self-launched ranks sharing the device)
if [ -n "$WITH_2RANK" ]; then
  timeout -k 10 900 python bench.py --gpus 2 > $O/bench_2rank_1gpu.log 2>&1 || { tail -20 $O/bench_2rank_1gpu.log; exit 1; }
  tail -1 $O/bench_2rank_1gpu.log | cut -c1-400
fi
echo done
