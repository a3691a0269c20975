# Round 3: how the headline encode responds to occupancy: the tree (6 waves
# per SIMD, VGPR-bound) against builds whose extra dynamic LDS leaves 5 and 4
# workgroups per CU (ECW_ASM_LDS_PAD), interleaved on the bench's tiled geometry.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/r03_occ_ab.log
: > $O
for args in "--chunk 8192 --split --pad 0 --stripes 8" "--stripes 4"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/kbench.py $args --rounds 4 ecwide_amd/libecwide.so build/variants/occ5.so build/variants/occ4.so 2>&1 | grep -v amdgpu >> $O || exit $?
done
cat $O
