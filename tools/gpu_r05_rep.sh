#!/bin/bash
# Round 5: the headline leg alone in six separate processes on one box (each a new
# allocation, so a new physical placement): the spread a single bench line can land
# in, on the final kernels.
# Run: gpurun -- 'bash tools/gpu_r05_rep.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05rep}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python bench.py --other-layout-steps 0 --configs4-steps 0 --shape-steps 0 --host-iters 0 --cpu-seconds 0 > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  python - $O/bench_$i.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print(d["value"], d["roofline"]["frac"], d["roofline"]["repair_frac"], d["verified"])
PY
done
