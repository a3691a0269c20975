#!/bin/bash
# Round 4: the k = 32 piece-size / CPU-baseline / tiled-K=2 script, then the
# encode-proxy XOR A/B, in one call.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/gpu_r04_k32.sh || exit $?
bash tools/gpu_r04_proxy.sh || exit $?
echo combo done
