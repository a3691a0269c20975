# Round 3: the 16-row asm tile (9-16 global rows in one pass): its parity
# tests first, then the GPU suite, then the two-pass round-2 build (base.so)
# against the tree on m > 8 shapes, interleaved on one allocation.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "more_than_8" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_nw4.log 2>&1 || { tail -40 gpurun_out/r03_pytest_nw4.log; exit 1; }
tail -3 gpurun_out/r03_pytest_nw4.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu_nw4.log 2>&1 || { tail -40 gpurun_out/r03_pytest_gpu_nw4.log; exit 1; }
tail -2 gpurun_out/r03_pytest_gpu_nw4.log
O=gpurun_out/r03_nw4_ab.log
: > $O
for args in "--code R --m 12 --k 128" "--code R --m 16 --k 128" "--code R --m 9 --k 128" "--m 10 --r 27 --k 128" "--code R --m 12 --k 128 --tables" "--code R --m 12 --k 200 --mib 16"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --stripes 4 --rounds 3 build/variants/base.so ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
