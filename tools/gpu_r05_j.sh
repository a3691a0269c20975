#!/bin/bash
# Round 5: the product with the three-slot ring under the write window against
# build/variants/ring2.so (-DECW_ASM_RING3=0 = the previous tile everywhere): the
# window-vs-off parity tests (every tail of the ring), then the whole-block
# layouts' encode through both builds in one process (block slab, pointer tables,
# split slab beside five tiled slabs).
# Build first: python tools/variants.py ring2=-DECW_ASM_RING3=0
# Run: gpurun -- 'bash tools/gpu_r05_j.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05j}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
V=${VARIANT:-build/variants/ring2.so}
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.log 2>&1 || { tail -40 $O/pytest_parity.log; exit 1; }
[ -n "${SKIP_TESTS:-}" ] || tail -2 $O/pytest_parity.log
for mode in "--check" "--tables"; do
  timeout -k 10 300 python -u tools/kbench.py --rounds 6 $mode ecwide_amd/libecwide.so $V ecwide_amd/libecwide.so@off > $O/kbench$mode.log 2>&1 || { tail -20 $O/kbench$mode.log; exit 1; }
  tail -4 $O/kbench$mode.log
done
timeout -k 10 500 python -u tools/repair_placement.py --scheds auto --enc-scheds auto --enc-libs $V > $O/placement.log 2>&1 || { tail -20 $O/placement.log; exit 1; }
tail -16 $O/placement.log
