# Round 3: the GPU suite on the current tree (software-pipelined asm rows,
# service yield/hold), then pipelined rows (pipe.so) vs the spill-free build
# without them (r03.so), interleaved on one allocation per shape.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03_pytest_gpu.log
grep -A1 "lifetime beside" gpurun_out/r03_pytest_gpu.log | head -3
V=build/variants
O=gpurun_out/r03_pipe_ab.log
echo "== tiled, bench shape" > $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $V/r03.so $V/pipe.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== tiled, configs[3] shape" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 256 --mib 8 --rounds 3 --chunk 8192 --split --pad 0 $V/r03.so $V/pipe.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== block slab (window on)" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --check $V/r03.so $V/pipe.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== pointer tables" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --tables $V/r03.so $V/pipe.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== pointer mode, blocks reversed (TAB asm tile)" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 4 --rounds 5 --ptr $V/r03.so $V/pipe.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== k=32 r=11 m=3 tiled" >> $O
timeout -k 10 300 python tools/kbench.py --k 32 --r 11 --m 3 --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $V/r03.so $V/pipe.so 2>&1 | grep -v amdgpu >> $O || exit $?
cat $O
