#!/bin/bash
# Round 5: K = 4 over PAIRS of the tiled slab's 8 KiB units (XorSplitPair) vs
# the K = 2 + window default, by the worst of five side-by-side tiled slabs,
# two processes; the tiled-repair schedule parity tests first.
# Run: gpurun -- 'bash tools/gpu_r05_f.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05f}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "tiled_repair_schedules or xor_schedules or full_size_tiled" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_sched.log 2>&1 || { tail -30 $O/pytest_sched.log; exit 1; }
tail -2 $O/pytest_sched.log
SCH="auto 1,0 4,0,11,64 4,0 4,1,11,64 4,0,11,32 2,1,11,64"
for i in 1 2; do
  timeout -k 10 400 python -u tools/repair_placement.py --split-at $((i * 2)) --scheds $SCH > $O/pair_placement_$i.log 2>&1 || { tail -20 $O/pair_placement_$i.log; exit 1; }
  tail -12 $O/pair_placement_$i.log
done
