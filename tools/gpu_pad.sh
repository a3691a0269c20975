cd $GRAFT_REPO_ROOT
V=build/variants
for pad in 0 4096 12288 69632 1060864 2097408; do
  echo "pad=$pad"; timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 3 --pad $pad $V/base.so $V/g512.so 2>&1 | grep -v amdgpu | tail -2 || exit $?
done
