cd $GRAFT_REPO_ROOT
V=build/variants
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --r 127 $V/base.so $V/ablate.so 2>&1 | grep -v amdgpu | tail -3 || exit $?
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --r 27 $V/base.so $V/ablate.so 2>&1 | grep -v amdgpu | tail -3 || exit $?
