# Round 3 profiles: the main leg of the default bench under the kernel tracer
# (only the main leg, so every encode_kernel_asm launch in the stats is one of
# the line's), the HBM-filling batch traced, FETCH_SIZE / WRITE_SIZE passes at
# the bench shape (tiled), the full default bench line, and ECWide-H's call
# patterns on both backends.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r03}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_$T
mkdir -p $O
V=build/variants
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $V/r03.so $V/ablate.so $V/ablate2.so 2>&1 | grep -v amdgpu > $O/ablate_ab.log || exit $?
cat $O/ablate_ab.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --other-layout-steps 0 --configs4-steps 0 --host-iters 0 > $O/bench_traced.log 2> $O/trace.log || exit $?
tail -1 $O/bench_traced.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/hbmfill -o run -- python3 $R/bench.py --hbm-fill --steps 10 --warmup 2 --cpu-seconds 0 --host-iters 0 > $O/hbmfill_bench.log 2> $O/hbmfill_trace.log || exit $?
tail -1 $O/hbmfill_bench.log | cut -c1-300
P="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --other-layout-steps 0 --configs4-steps 0 --host-iters 0 --no-verify"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_tiled -o run -- $P > $O/fetch_tiled.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_tiled -o run -- $P > $O/write_tiled.log 2>&1 || exit $?
cd $R
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || exit $?
tail -1 $O/bench_default.log | cut -c1-300
bash tools/gpu_shim.sh > $O/shim.log 2>&1 || { tail -5 $O/shim.log; exit 1; }
cp gpurun_out/shim_bench.log $O/shim_bench.log
timeout -k 10 300 python bench.py --small-calls > $O/bench_small.log 2>&1 || { tail -20 $O/bench_small.log; exit 1; }
find $O -name "*stats.csv" | head
echo done
