# Round 3: the 8-row asm tile with interleaved hi/lo table entries (one shift
# per data dword) and v_bitop3 address builds (the tree) against HEAD before
# the change (head.so): the GPU suite first, then interleaved A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu_nw2b.log 2>&1 || { tail -40 gpurun_out/r03_pytest_gpu_nw2b.log; exit 1; }
tail -2 gpurun_out/r03_pytest_gpu_nw2b.log
O=gpurun_out/r03_nw2b_ab.log
: > $O
for args in "--code R --m 8 --k 128" "--code R --m 5 --k 128" "--m 6 --r 27 --k 128" "--m 8 --r 27 --k 128 --literal" "--code R --m 3 --k 128"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --stripes 4 --rounds 4 build/variants/head.so ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
