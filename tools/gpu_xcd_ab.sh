# XCD-contiguous tile mapping (-DECW_XCD_REMAP=1) vs round-robin, same allocation,
# 8 MiB blocks at a mid-size and an HBM-filling slab
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=build/variants/base.so,build/variants/xcd.so
timeout -k 10 300 python -u tools/layout_ab.py --mib 8 --stripes 32 --rounds 5 --iters 5 --variants tiled:8192:0 --libs $L > gpurun_out/xcd_ab_32.log 2>&1 || exit 1
cat gpurun_out/xcd_ab_32.log
timeout -k 10 400 python -u tools/layout_ab.py --mib 8 --stripes 240 --rounds 4 --iters 3 --variants tiled:8192:0 --libs $L > gpurun_out/xcd_ab_240.log 2>&1 || exit 1
cat gpurun_out/xcd_ab_240.log
timeout -k 10 300 python -u tools/layout_ab.py --mib 64 --stripes 8 --rounds 5 --iters 5 --variants tiled:8192:0,blocks:4096 --libs $L > gpurun_out/xcd_ab_64m.log 2>&1 || exit 1
cat gpurun_out/xcd_ab_64m.log
