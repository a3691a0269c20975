# Round 3 end-to-end check on one box: the GPU suite (with the lifetime
# test's numbers), smoke, the default bench, configs[3], the N=2 self-launch,
# the driver's torchrun form at N=2 / 4, then the split slab's write-window A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_service.py -k lifetime -x -s -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_lifetime.log 2>&1 || { tail -30 gpurun_out/r03_lifetime.log; exit 1; }
grep "lifetime beside" gpurun_out/r03_lifetime.log
bash tools/gpu_check.sh || exit $?
bash tools/gpu_ranks.sh || exit $?
V=build/variants
echo "== split slab (whole blocks, parities apart), window off / on" > gpurun_out/r03_split_window.log
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 6 --chunk 67108864 --split --pad 0 $V/pipe.so@off $V/pipe.so@on 2>&1 | grep -v amdgpu >> gpurun_out/r03_split_window.log || exit $?
cat gpurun_out/r03_split_window.log
