#!/bin/bash
# Round 5, first check of the refactored tree (kernels split into four
# translation units, ecw_set_schedule instead of per-launch getenv, K = 2 XOR
# skew built in): smoke, the GPU suite, then the tiled-repair placement study
# (tools/repair_placement.py: 5 tiled slabs + 1 split slab side by side, every
# XOR schedule on every slab, two processes with the split slab at different
# positions), then the default bench line.
# Run: gpurun -- 'bash tools/gpu_r05_a.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05a}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 400 python -u tools/repair_placement.py --split-at 0 > $O/placement_1.log 2>&1 || { tail -20 $O/placement_1.log; exit 1; }
tail -16 $O/placement_1.log
timeout -k 10 400 python -u tools/repair_placement.py --split-at 5 > $O/placement_2.log 2>&1 || { tail -20 $O/placement_2.log; exit 1; }
tail -16 $O/placement_2.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-400
