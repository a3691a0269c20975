#!/bin/bash
# Round 5: check of the tree with the tiled encode's write window (2^11 / 32 with
# the three-slot ring): smoke, the GPU suite, the placement study (auto = the new
# default) in one process, the default bench.
# Run: gpurun -- 'bash tools/gpu_r05_m.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05m}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 500 python -u tools/repair_placement.py --split-at 3 --scheds auto --enc-scheds auto off 11,32 > $O/placement.log 2>&1 || { tail -20 $O/placement.log; exit 1; }
tail -6 $O/placement.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
