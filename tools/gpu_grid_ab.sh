# encode grid size / launch windows (ECW_GRID_PER_CU, ECW_COHORT_TILES) on one
# allocation: HBM-filling slab of 8 MiB blocks and the bench shape
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
L=$(for v in ${LIBS:-base g1k g2k coh64k coh32k}; do printf 'build/variants/%s.so,' $v; done); L=${L%,}
timeout -k 10 400 python -u tools/layout_ab.py --mib 8 --stripes 240 --rounds 3 --iters 3 --variants tiled:8192:0 --libs $L > gpurun_out/grid_ab_240.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/grid_ab_240.log
timeout -k 10 300 python -u tools/layout_ab.py --mib 64 --stripes 8 --rounds 5 --iters 5 --variants tiled:8192:0 --libs $L > gpurun_out/grid_ab_64m.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/grid_ab_64m.log
