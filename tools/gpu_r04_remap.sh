#!/bin/bash
# Round 4: per-XCD contiguous tile order (ECW_XCD_REMAP=1: a CU's resident
# workgroups take tiles 32 apart instead of 256, sharing more translations)
# for the whole-block layouts, whose encode keeps the UTCL2 93-96 % busy
# (profiles/r04b_repair_pmc_summary.txt); two processes, reversed order.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/repair_ab.py --stripes 4 --rounds 3 --encode --enc-windows auto auto+r off+r \
  --placements sep,split,carved4k,tiled --scheds auto auto+r > gpurun_out/r04_remap_1.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --stripes 4 --rounds 3 --encode --enc-windows auto auto+r off+r \
  --placements tiled,carved4k,split,sep --scheds auto auto+r > gpurun_out/r04_remap_2.log 2>&1
