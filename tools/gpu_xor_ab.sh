cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=build/variants
timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_xor.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_xor.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_xor.log
timeout -k 10 400 python -u tools/layout_ab.py --rounds 5 --iters 5 --variants blocks:4096,tiled:8192:0 --libs $V/base.so,$V/w4.so,$V/w8.so,$V/w16.so,$V/wall.so > gpurun_out/xor_window_ab.log 2>&1 || exit 1
cat gpurun_out/xor_window_ab.log
