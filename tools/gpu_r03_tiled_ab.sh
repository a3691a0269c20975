# Round 3: what is left on the spill-free tiled encode. Interleaved on one
# allocation (tiled geometry): write window off / on / other periods, the
# math-free build, no table staging, one launch, nt-only stores.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=build/variants
O=gpurun_out/r03_tiled_ab.log
timeout -k 10 400 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 \
  $V/r03.so@off $V/r03.so@on $V/r03.so@10,32 $V/r03.so@12,128 $V/r03.so@11,128 $V/r03.so@12,64 \
  $V/ablate.so@off $V/ablate.so@on $V/nostage.so@off $V/nostage.so@on $V/one.so@off $V/one.so@on \
  $V/ring_stnt.so@on 2>&1 | grep -v amdgpu > $O || exit $?
echo "== split slab (whole blocks, parities apart)" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 67108864 --split --pad 0 $V/r03.so@off $V/r03.so@on 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== configs[3] shape: 256 x 8 MiB tiled (ticket launch)" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 256 --mib 8 --rounds 3 --chunk 8192 --split --pad 0 $V/r03.so@off $V/r03.so@on 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== k=32 r=11 m=3 64 MiB x8 tiled (configs[0] shape)" >> $O
timeout -k 10 300 python tools/kbench.py --k 32 --r 11 --m 3 --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $V/r03.so@off $V/r03.so@on 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== k=32 r=8 m=2 16 MiB x32 tiled (configs[1] shape)" >> $O
timeout -k 10 300 python tools/kbench.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --rounds 5 --chunk 8192 --split --pad 0 $V/r03.so@off $V/r03.so@on 2>&1 | grep -v amdgpu >> $O || exit $?
cat $O
