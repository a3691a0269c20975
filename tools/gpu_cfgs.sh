# bench.py at BASELINE configs[1] (k=32, 4 groups, m=2, 16 MiB) and the default
# scheme.ini shape (configs[0]: k=32, r=11, m=3, 64 MiB), plus literal-mode A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python bench.py --k 32 --m 2 --r 8 --block-mib 16 --stripes 32 --cpu-seconds 0 --verify > gpurun_out/bench_cfg2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --k 32 --m 3 --r 11 --block-mib 64 --stripes 8 --cpu-seconds 0 --verify > gpurun_out/bench_cfg1.log 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 ecwide_amd/libecwide.so > gpurun_out/kb_xor.log 2>&1 || exit $?
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 3 --literal ecwide_amd/libecwide.so > gpurun_out/kb_literal.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cfg2.log | cut -c1-300; tail -1 gpurun_out/bench_cfg1.log | cut -c1-300; tail -1 gpurun_out/kb_xor.log; tail -1 gpurun_out/kb_literal.log
