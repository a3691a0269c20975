cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
nproc > gpurun_out/host.txt; lscpu >> gpurun_out/host.txt 2>&1; rocm-smi --showmeminfo vram >> gpurun_out/host.txt 2>&1
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 400 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --verify > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo "prof rc=$?"
