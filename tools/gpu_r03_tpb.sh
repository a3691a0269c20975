# Round 3: the 16-row asm kernel with 2-tile workgroups (the tree) against
# 1-tile workgroups (tpb1.so): parity tests of m > 8 first, then the GPU
# suite, then interleaved A/B on m > 8 shapes (k = 128 and the 100 KiB
# tables of k = 200).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "more_than_8 or ticket" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_tpb.log 2>&1 || { tail -40 gpurun_out/r03_pytest_tpb.log; exit 1; }
tail -3 gpurun_out/r03_pytest_tpb.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu_tpb.log 2>&1 || { tail -40 gpurun_out/r03_pytest_gpu_tpb.log; exit 1; }
tail -2 gpurun_out/r03_pytest_gpu_tpb.log
O=gpurun_out/r03_tpb_ab.log
: > $O
for args in "--code R --m 12 --k 128" "--code R --m 16 --k 128" "--m 10 --r 27 --k 128" "--code R --m 12 --k 200 --mib 16" "--code R --m 12 --k 64"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --stripes 4 --rounds 3 build/variants/tpb1.so ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
