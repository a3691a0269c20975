#!/bin/bash
# Round 5: timeline of the host-resident pipeline (kernel + memory-copy trace).
# Run: gpurun -- 'bash tools/gpu_r05_tl.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05tl}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 300 python3 tools/host_timeline.py > $O/plain.log 2>&1 || { tail -20 $O/plain.log; exit 1; }
cat $O/plain.log | grep iter
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/host_timeline.py > $O/traced.log 2>&1 || { tail -20 $O/traced.log; exit 1; }
grep iter $O/traced.log
ls $O/trace
