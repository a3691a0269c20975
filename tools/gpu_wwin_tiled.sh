# GPU suite, then the tiled slab's write-window A/B (more rounds, several periods).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_wwin.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_wwin.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_wwin.log
L=ecwide_amd/libecwide.so
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $L@off $L@on $L@10,32 $L@12,128 $L@11,32 2>&1 | grep -v amdgpu > gpurun_out/wwin_tiled.log || exit $?
cat gpurun_out/wwin_tiled.log
