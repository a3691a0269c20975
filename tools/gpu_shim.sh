# ECWide-H's call patterns through ISA-L's API on both backends: the GPU
# engine behind libecw_isal.so and the CPU (the oracle's AVX2 port of ISA-L's
# kernels), synchronous 4 KiB calls, the per-chunk call sequence, and the
# proxy's own concurrency (one thread per role, then 2 and 4 per role).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
gcc -O2 -o /tmp/shim_bench tools/csrc/shim_bench.c -ldl -lpthread || exit 1
O=gpurun_out/shim_bench.log
: > $O
for be in gpu cpu; do
  for t in 1 4 16; do timeout -k 10 120 /tmp/shim_bench $be calls $t 2000 >> $O 2>&1 || exit $?; done
  for t in 1 4; do timeout -k 10 120 /tmp/shim_bench $be seq $t 1000 >> $O 2>&1 || exit $?; done
  for t in 1 2 4; do timeout -k 10 120 /tmp/shim_bench $be proxy $t 2000 >> $O 2>&1 || exit $?; done
done
cat $O
