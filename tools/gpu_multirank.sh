# Rehearse the N>1 bench path on a 1-GPU box: 2 ranks share cuda:0 (gloo for
# the timing collective); weak (2 stripes each) and strong (3 stripes total).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 400 $R --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 2 > gpurun_out/bench_2rank.log 2>&1 || exit $?
tail -1 gpurun_out/bench_2rank.log | cut -c1-400
timeout -k 10 400 $R --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 3 --strong > gpurun_out/bench_2rank_strong.log 2>&1 || exit $?
tail -1 gpurun_out/bench_2rank_strong.log | cut -c1-600
timeout -k 10 400 $R --master-port 29535 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 1 --strong > gpurun_out/bench_2rank_columns.log 2>&1 || exit $?
tail -1 gpurun_out/bench_2rank_columns.log | cut -c1-700
