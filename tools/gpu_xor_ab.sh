# A/B of XOR-repair variants (build/variants/*.so, tools/variants.py) on one
# allocation, block and tiled slab: LIBS="a b c" bash tools/gpu_xor_ab.sh
# (PYTEST=1 runs the GPU parity tests on the in-tree build first)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
if [ -n "$PYTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests -q -x -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_xor.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_xor.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_xor.log
fi
L=$(for v in ${LIBS:-base w4 w8 w16 wall}; do printf 'build/variants/%s.so,' $v; done)
timeout -k 10 400 python -u tools/layout_ab.py --rounds ${ROUNDS:-5} --iters 5 --variants ${VARIANTS:-blocks:4096,tiled:8192:0} --libs ${L%,} > gpurun_out/xor_ab.log 2>&1 || exit 1
cat gpurun_out/xor_ab.log
