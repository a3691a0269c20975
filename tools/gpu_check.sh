# Parity suite + smoke + the bench at N=1 (default), configs[3] and the
# N=2 self-launch rehearsed on one GPU. Each GPU step has its own limit; the
# script stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$T.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$T.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$T.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_$T.log 2>&1 || { tail -20 gpurun_out/bench_$T.log; exit 1; }
tail -1 gpurun_out/bench_$T.log | cut -c1-300
timeout -k 10 400 python bench.py --hbm-fill --steps 10 --warmup 2 --cpu-seconds 0 > gpurun_out/bench_hbmfill_$T.log 2>&1 || { tail -20 gpurun_out/bench_hbmfill_$T.log; exit 1; }
tail -1 gpurun_out/bench_hbmfill_$T.log | cut -c1-300
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_2gpu_$T.log 2>&1 || { tail -20 gpurun_out/bench_2gpu_$T.log; exit 1; }
tail -1 gpurun_out/bench_2gpu_$T.log | cut -c1-300
