cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_exp.sh > gpurun_out/exp5.log 2>&1 || exit $?
timeout -k 10 240 python tools/kbench.py --stripes 8 --rounds 3 --code R build/variants/noasm.so build/variants/asm.so 2>&1 | grep -v amdgpu >> gpurun_out/exp5.log
