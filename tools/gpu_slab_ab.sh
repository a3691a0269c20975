# Bench-step A/B of the tiled and split slabs in one process (tools/slab_ab.py),
# twice (two allocations), plus the k=32 shape.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
for i in 1 2; do
timeout -k 10 300 python tools/slab_ab.py >> gpurun_out/slab_ab_$T.log 2>&1 || { tail -20 gpurun_out/slab_ab_$T.log; exit 1; }
done
timeout -k 10 300 python tools/slab_ab.py --k 32 --m 2 --r 8 --mib 16 --stripes 32 >> gpurun_out/slab_ab_$T.log 2>&1 || exit $?
cat gpurun_out/slab_ab_$T.log
