# Rank rehearsal on one GPU: the driver's own torchrun command line for N=2
# and N=4 ranks sharing cuda:0, plus the JNI GPU tests. Each step has its own
# limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r03}
timeout -k 10 300 python -u -m pytest tests/test_jni.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_jni_$T.log 2>&1 || { tail -30 gpurun_out/pytest_jni_$T.log; exit 1; }
tail -1 gpurun_out/pytest_jni_$T.log
# N ranks share one GPU here: 8 stripes of 64 MiB per rank (the default) for
# N=2 (2 x 68 GiB), 2 per rank for N=4, so the slabs fit one card together
for N in 2 4; do
  S=$([ $N -le 2 ] && echo 8 || echo 2)
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus $N --stripes $S --steps 10 --warmup 2 > gpurun_out/bench_torchrun_n${N}_$T.log 2>&1 || { tail -20 gpurun_out/bench_torchrun_n${N}_$T.log; exit 1; }
  grep '^{' gpurun_out/bench_torchrun_n${N}_$T.log | tail -1 | cut -c1-400
done
