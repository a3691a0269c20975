# The small-stripe request service: its tests, the ISA-L shim callers (C
# pthreads) and the --small-calls bench line with its CPU baseline.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py tests/test_isal_shim.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_service_$T.log 2>&1 || { tail -40 gpurun_out/pytest_service_$T.log; exit 1; }
tail -3 gpurun_out/pytest_service_$T.log
cd tools/csrc && gcc -O2 -o /tmp/shim_bench shim_bench.c -ldl -lpthread || exit 1
cd $GRAFT_REPO_ROOT
for t in 1 4 16; do timeout -k 10 120 /tmp/shim_bench gpu calls $t 2000 >> gpurun_out/shim_bench_$T.log 2>&1 || exit $?; done
for t in 1 4; do timeout -k 10 120 /tmp/shim_bench gpu seq $t 1000 >> gpurun_out/shim_bench_$T.log 2>&1 || exit $?; done
ECW_ISAL_BATCH=1 timeout -k 10 120 /tmp/shim_bench gpu calls 4 2000 >> gpurun_out/shim_bench_$T.log 2>&1 || exit $?
ECW_SERVICE=0 timeout -k 10 120 /tmp/shim_bench gpu calls 1 2000 >> gpurun_out/shim_bench_$T.log 2>&1 || exit $?
ECW_SERVICE=0 timeout -k 10 120 /tmp/shim_bench gpu calls 4 2000 >> gpurun_out/shim_bench_$T.log 2>&1 || exit $?
cat gpurun_out/shim_bench_$T.log
timeout -k 10 300 python bench.py --small-calls > gpurun_out/bench_small_$T.log 2>&1 || { tail -20 gpurun_out/bench_small_$T.log; exit 1; }
tail -1 gpurun_out/bench_small_$T.log
