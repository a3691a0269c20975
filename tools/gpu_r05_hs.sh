#!/bin/bash
# Round 5: the host pipeline's host -> HBM copies on two streams (the product)
# against one (build/variants/in1.so = -DECW_HOST_IN_STREAMS=1): the host-path GPU
# tests, then tools/host_ab.py (same pinned blocks, interleaved), twice.
# Build first: python tools/variants.py in1=-DECW_HOST_IN_STREAMS=1
# Run: gpurun -- 'bash tools/gpu_r05_hs.sh'
set -uo pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r05hs}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "host or pinned or chunk or jni or isal or service or c_abi" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_host.log 2>&1 || { tail -40 $O/pytest_host.log; exit 1; }
tail -2 $O/pytest_host.log
for i in 1 2; do
  timeout -k 10 400 python -u tools/host_ab.py build/variants/in1.so --rounds 6 > $O/host_ab_$i.log 2>&1 || { tail -20 $O/host_ab_$i.log; exit 1; }
  tail -3 $O/host_ab_$i.log
done
