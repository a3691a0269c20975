# Round 3: parked local parities (78 VGPRs, 6 waves/SIMD) against mid-tile
# local stores (57 VGPRs, 8 waves/SIMD), interleaved on one allocation.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=build/variants
O=gpurun_out/r03_park_ab.log
echo "== tiled, bench shape" > $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $V/r03.so $V/nopark.so $V/nopark8.so $V/ablate.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== tiled, configs[3] shape (256 x 8 MiB)" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 256 --mib 8 --rounds 3 --chunk 8192 --split --pad 0 $V/r03.so $V/nopark.so $V/nopark8.so 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== block slab" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 $V/r03.so $V/nopark.so $V/nopark8.so 2>&1 | grep -v amdgpu >> $O || exit $?
cat $O
