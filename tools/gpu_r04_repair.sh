#!/bin/bash
# Round 4: the reworked XOR kernel and service on the GPU (service + XOR parity
# tests), then CL repair over separately allocated blocks vs the slabs with the
# XOR schedules A/B (tools/repair_ab.py), two processes with the allocation
# order reversed. Run: gpurun -- 'bash tools/gpu_r04_repair.sh'
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
LIB=${LIB:-build/variants/skewall.so}
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_service.py \
    tests/test_gpu_parity.py -k "service or xor or repair or decode or Service" > gpurun_out/r04_pytest_xor_service.log 2>&1
fi
timeout -k 10 300 python -u tools/repair_ab.py --lib "$LIB" --stripes 4 --encode \
  > gpurun_out/r04_repair_ab_1.log 2>&1
timeout -k 10 300 python -u tools/repair_ab.py --lib "$LIB" --stripes 4 --encode \
  --placements carved4k,carved0,sep,split,tiled > gpurun_out/r04_repair_ab_2.log 2>&1
