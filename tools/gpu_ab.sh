# A/B of build/variants/*.so on one GPU: CL(128,27,3) 64 MiB x8 stripes, then
# any extra kbench invocations given as arguments ("--k 32 --r 8 ..." strings).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/ab.log}
V=$(ls build/variants/*.so | sort)
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --check $V 2>&1 | grep -v amdgpu > $OUT || exit $?
for extra in "$@"; do
  timeout -k 10 300 python tools/kbench.py --rounds 3 $extra $V 2>&1 | grep -v amdgpu >> $OUT || exit $?
done
