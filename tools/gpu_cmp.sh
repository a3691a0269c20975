cd $GRAFT_REPO_ROOT
V=build/variants
K="timeout -k 10 240 python tools/kbench.py --stripes 8 --rounds 3 $V/base.so"
$K 2>&1 | grep -v amdgpu | tail -2 &&
$K --chunk 1048576 --pad 0 2>&1 | grep -v amdgpu | tail -2 &&
$K --chunk 262144 --pad 0 2>&1 | grep -v amdgpu | tail -2 &&
$K --chunk 65536 --pad 0 2>&1 | grep -v amdgpu | tail -2 &&
$K --chunk 65536 --pad 4096 2>&1 | grep -v amdgpu | tail -2 &&
$K --chunk 16384 --pad 0 2>&1 | grep -v amdgpu | tail -2
