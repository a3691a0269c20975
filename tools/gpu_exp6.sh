cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/gpu_exp.sh > gpurun_out/exp6.log 2>&1 || exit $?
timeout -k 10 240 python tools/kbench.py --stripes 8 --rounds 3 --code R build/variants/asm.so build/variants/asmnt.so build/variants/asmntst.so 2>&1 | grep -v amdgpu >> gpurun_out/exp6.log
