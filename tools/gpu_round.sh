# One GPU round: parity tests, smoke, bench, rocprof kernel stats, PMC traffic,
# host-resident (PCIe) rate. Every GPU step has its own time limit; the
# script stops at the first failure. The committed bench line
# (gpurun_out/bench.log) comes from the SAME process rocprofv3 traced, so the
# bench's event timing and the rocprof kernel average describe the same launches.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
TAG=${TAG:-r01}
R=$GRAFT_REPO_ROOT
nproc > gpurun_out/host.txt; lscpu >> gpurun_out/host.txt 2>&1
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --verify > gpurun_out/bench_unprofiled.log 2>&1 || exit $?
tail -1 gpurun_out/bench_unprofiled.log
cd /tmp
# the default bench under the kernel tracer (other-layout leg off: it launches the same kernels)
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --verify --other-layout-steps 0 > $R/gpurun_out/bench.log 2> $R/gpurun_out/prof.log || exit $?
tail -1 $R/gpurun_out/bench.log
P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- $P > $R/gpurun_out/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- $P > $R/gpurun_out/pmc2.log 2>&1 || exit $?
echo "profiles done"
cd $R && timeout -k 10 400 python bench.py --host-resident --steps 12 > gpurun_out/bench_host.log 2>&1 || exit $?
tail -1 gpurun_out/bench_host.log
