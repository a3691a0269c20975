cd $GRAFT_REPO_ROOT
V=build/variants
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 4 --check $V/base.so $V/lds.so $V/nts.so $V/w6.so $V/w6lds.so 2>&1 | grep -v amdgpu | tail -6 || exit $?
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --code R $V/base.so $V/w6.so 2>&1 | grep -v amdgpu | tail -3 || exit $?
