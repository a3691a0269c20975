cd $GRAFT_REPO_ROOT
V=build/variants
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --check $V/base.so $V/g512.so $V/coh1280.so $V/coh2560.so $V/coh5120.so $V/coh16k.so 2>&1 | grep -v amdgpu | tail -7 || exit $?
for pad in 0 12288 69632 2097408; do
  echo "pad=$pad"; timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 3 --pad $pad $V/base.so 2>&1 | grep -v amdgpu | tail -1 || exit $?
done
