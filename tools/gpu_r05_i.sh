#!/bin/bash
# Round 5: the three-slot ring (build/variants/ring3.so) on the whole-block layouts
# and at the k = 32 BASELINE shapes: block slab and pointer tables over separate
# allocations at CL(128, 27, 3) (tools/kbench.py, both builds interleaved in one
# process), then five tiled slabs + one split slab at configs[1] / configs[0]'s shapes.
# Run: gpurun -- 'bash tools/gpu_r05_i.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05i}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
V=${VARIANT:-build/variants/ring3.so}
timeout -k 10 300 python -u tools/kbench.py --rounds 6 --check ecwide_amd/libecwide.so $V > $O/kbench_block.log 2>&1 || { tail -20 $O/kbench_block.log; exit 1; }
tail -3 $O/kbench_block.log
timeout -k 10 300 python -u tools/kbench.py --rounds 6 --tables ecwide_amd/libecwide.so $V > $O/kbench_tables.log 2>&1 || { tail -20 $O/kbench_tables.log; exit 1; }
tail -3 $O/kbench_tables.log
timeout -k 10 400 python -u tools/repair_placement.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --scheds auto --enc-scheds auto --enc-libs $V > $O/placement_cfg1.log 2>&1 || { tail -20 $O/placement_cfg1.log; exit 1; }
tail -8 $O/placement_cfg1.log
timeout -k 10 400 python -u tools/repair_placement.py --k 32 --r 11 --m 3 --mib 64 --stripes 8 --scheds auto --enc-scheds auto --enc-libs $V > $O/placement_cfg0.log 2>&1 || { tail -20 $O/placement_cfg0.log; exit 1; }
tail -8 $O/placement_cfg0.log
