# A/B of build/variants/*.so across block sizes (CL k=128, ~68 GiB slabs)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=$(ls build/variants/*.so | sort)
: > gpurun_out/ab_sizes.log
for ms in "4 128" "16 32" "32 16"; do set -- $ms
  timeout -k 10 300 python tools/kbench.py --mib $1 --stripes $2 --rounds 3 --iters 3 $V 2>&1 | grep -v amdgpu >> gpurun_out/ab_sizes.log || exit $?
done
