cd $GRAFT_REPO_ROOT
V=build/variants
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --check $V/base.so $V/x4.so $V/x16.so $V/xg64.so $V/b512.so 2>&1 | grep -v amdgpu | tail -6 || exit $?
