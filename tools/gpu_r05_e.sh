#!/bin/bash
# Round 5: what NUMA-local host staging buys (tools/host_numa_ab.py: the same
# host-resident encode + repair with the pinned stripe on every NUMA node in
# turn, interleaved), and the GPU tests of the staging.
# Run: gpurun -- 'bash tools/gpu_r05_e.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05e}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
lscpu > $O/lscpu.txt 2>&1; numactl -H > $O/numactl.txt 2>&1 || true
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pinned_host or host_pipeline" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_host.log 2>&1 || { tail -30 $O/pytest_host.log; exit 1; }
tail -2 $O/pytest_host.log
timeout -k 10 600 python -u tools/host_numa_ab.py --rounds 4 > $O/host_numa_ab.log 2>&1 || { tail -20 $O/host_numa_ab.log; exit 1; }
cat $O/host_numa_ab.log
