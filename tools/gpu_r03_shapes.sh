# Round 3: the GPU suite on the current tree (16-row tile, early ring loads),
# the early-load A/B (noearly.so vs early.so) on the bench shapes, then
# off-config encode shapes on round 2's build (base.so) and the current one.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r03_pytest_gpu.log
V=build/variants
O=gpurun_out/r03_early_ab.log
echo "== tiled, bench shape" > $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $V/noearly.so $V/early.so $V/ablate.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== tiled, configs[3] shape" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 256 --mib 8 --rounds 3 --chunk 8192 --split --pad 0 $V/noearly.so $V/early.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== block slab" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 $V/noearly.so $V/early.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== k=32 r=8 m=2 16 MiB x32 tiled" >> $O
timeout -k 10 300 python tools/kbench.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --rounds 5 --chunk 8192 --split --pad 0 $V/noearly.so $V/early.so 2>&1 | grep -v amdgpu >> $O || exit $?
cat $O
O=gpurun_out/r03_shapes.log
: > $O
for args in "--code R --m 12 --k 128" "--code R --m 16 --k 128" "--code R --m 5 --k 128" "--code R --m 8 --k 128" "--m 6 --r 27 --k 128" "--m 4 --r 40 --k 200 --mib 16" "--code R --m 3 --k 128"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --stripes 4 --rounds 3 $V/base.so $V/early.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
