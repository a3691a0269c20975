#!/bin/bash
# Round 4: 2-tile workgroups (-DECW_ASM_TPB1=2: 8 waves share one LDS copy of the
# tables and take two adjacent 4 KiB tiles) for the pointer-table encode, with
# the per-XCD order, against the product, same blocks (tools/kbench.py --tables).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/kbench.py --tables --stripes 8 --rounds 5 ecwide_amd/libecwide.so build/variants/tpb2.so \
  > gpurun_out/r04_tpb2_tables.log 2>&1
timeout -k 10 300 python -u tools/kbench.py --tables --stripes 8 --rounds 5 build/variants/tpb2.so ecwide_amd/libecwide.so \
  > gpurun_out/r04_tpb2_tables_rev.log 2>&1
