# A/B of build/variants/*.so at the HBM-filling shape (256 stripes x 136 blocks of 8 MiB)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python tools/kbench.py --mib 8 --stripes 256 --rounds 3 --iters 3 $(ls build/variants/*.so | sort) 2>&1 | grep -v amdgpu > gpurun_out/ab_fill.log || exit $?
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 $(ls build/variants/*.so | sort) 2>&1 | grep -v amdgpu >> gpurun_out/ab_fill.log
