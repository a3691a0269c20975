# Block-layout experiments (tilebench), the counter list, CPU baselines on
# the box's cores and the k=32 configuration bench lines.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
hipcc --offload-arch=gfx950 -O3 tools/csrc/tilebench.hip -o /tmp/tilebench || exit 1
timeout -k 10 300 /tmp/tilebench 5 > gpurun_out/tilebench_$T.log 2>&1 || exit $?
cat gpurun_out/tilebench_$T.log
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc_list_$T.txt 2>&1 || echo "counter list rc=$?"
grep -i -c "utcl\|tlb" gpurun_out/pmc_list_$T.txt
timeout -k 10 600 python tools/cpu_baseline.py > gpurun_out/cpu_baselines_$T.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --k 32 --m 3 --r 11 --block-mib 64 --stripes 8 --no-verify > gpurun_out/bench_cfg0_$T.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --k 32 --m 2 --r 8 --block-mib 16 --stripes 32 > gpurun_out/bench_cfg1_$T.log 2>&1 || exit $?
echo done
