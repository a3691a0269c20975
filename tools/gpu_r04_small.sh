#!/bin/bash
# Round 4: ECWide-H's synchronous small calls (bench.py --small-calls): per-call
# latency, and the 4-call mix with the service's hit rate and p50 / p99.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --small-calls --small-calls-n 3000 > gpurun_out/r04_bench_small_calls.log 2>&1
tail -1 gpurun_out/r04_bench_small_calls.log | cut -c1-400
