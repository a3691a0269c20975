# BASELINE configs[3]: 256 stripes filling HBM — bench line, rocprof kernel
# stats, PMC FETCH_SIZE / WRITE_SIZE passes (separate runs).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/hbmfill && export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/hbmfill
timeout -k 10 300 python bench.py --hbm-fill --steps 10 --warmup 2 --cpu-seconds 0 --verify > $O/bench.log 2>&1 || exit $?
tail -1 $O/bench.log
cd /tmp
P="python3 $GRAFT_REPO_ROOT/bench.py --hbm-fill --steps 5 --warmup 1 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- $P > $O/prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- $P > $O/pmc1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- $P > $O/pmc2.log 2>&1 || exit $?
echo done
