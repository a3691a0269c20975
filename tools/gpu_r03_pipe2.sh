# Round 3: the 8-row asm tile with rows pipelined across row boundaries and
# early ring loads (pipe2.so = the tree) against the round-3 unpipelined rows
# (nopipe2.so), interleaved on one allocation; parity tests of the 5-8-row and
# >8-row paths first.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_pipe2.log 2>&1 || { tail -30 gpurun_out/r03_pytest_pipe2.log; exit 1; }
tail -1 gpurun_out/r03_pytest_pipe2.log
V=build/variants
O=gpurun_out/r03_pipe2_ab.log
: > $O
for args in "--code R --m 8 --k 128" "--code R --m 5 --k 128" "--m 6 --r 27 --k 128" "--code R --m 12 --k 128" "--m 6 --r 27 --k 128 --tables" "--code R --m 3 --k 128"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --stripes 4 --rounds 4 $V/nopipe2.so $V/pipe2.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
