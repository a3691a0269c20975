# Round 3: <= 4-row asm kernel with 2-tile (512-thread) workgroups sharing one
# LDS copy of the tables (tpb2.so) against the tree (1 tile per workgroup):
# parity on the tiled geometry first (kbench --check on the block slab), then
# interleaved A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03_tpb1_ab.log
: > $O
for args in "--check --stripes 2" "--chunk 8192 --split --pad 0 --stripes 8" "--stripes 4" "--tables --stripes 8"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --rounds 4 ecwide_amd/libecwide.so build/variants/tpb2.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
