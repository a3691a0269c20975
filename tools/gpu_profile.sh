# Round profiles: the default bench under the kernel tracer (its own line and
# the rocprof averages of the same launches), FETCH_SIZE / WRITE_SIZE passes
# (separate runs) at the bench shape for the tiled and split slabs, and the
# HBM-filling batch traced.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$T
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 > $O/bench.log 2> $O/trace.log || exit $?
tail -1 $O/bench.log | cut -c1-200
for L in tiled split; do
P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0 --no-verify --layout $L"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$L -o run -- $P > $O/fetch_$L.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$L -o run -- $P > $O/write_$L.log 2>&1 || exit $?
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hbmfill -o run -- python3 $R/bench.py --hbm-fill --steps 10 --warmup 2 --cpu-seconds 0 > $O/hbmfill_bench.log 2> $O/hbmfill_trace.log || exit $?
tail -1 $O/hbmfill_bench.log | cut -c1-200
find $O -name "*.csv" | head -50
echo done
