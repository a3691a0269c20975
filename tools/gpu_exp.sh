# Generic interleaved A/B of build/variants/*.so (args: extra kbench flags).
cd $GRAFT_REPO_ROOT
V=build/variants
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --check "$@" $(ls $V/*.so | sort) 2>&1 | grep -v amdgpu
