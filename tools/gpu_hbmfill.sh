# BASELINE configs[3]: 256 stripes filling HBM — the bench line from the process
# rocprofv3 traced (kernel stats of the same launches), then PMC FETCH_SIZE /
# WRITE_SIZE passes (separate runs).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/hbmfill && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/hbmfill
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --hbm-fill --steps 10 --warmup 2 --cpu-seconds 0 --host-iters 0 --verify > $O/bench.log 2> $O/prof.log || exit $?
tail -1 $O/bench.log
P="python3 $GRAFT_REPO_ROOT/bench.py --hbm-fill --steps 5 --warmup 1 --cpu-seconds 0 --host-iters 0 --no-verify"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $P > $O/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $P > $O/pmc2.log 2>&1 || exit $?
echo done
