# C pthread callers of libecw_isal.so (ECWide-H-style synchronous 4 KiB calls)
cd $GRAFT_REPO_ROOT/tools/csrc && gcc -O2 -o shim_bench shim_bench.c -L../../ecwide_amd -lecw_isal -lpthread -Wl,-rpath,$GRAFT_REPO_ROOT/ecwide_amd || exit 1
for t in 1 4 16; do timeout -k 10 120 ./shim_bench $t 400 || exit $?; done
ECW_ISAL_BATCH=0 timeout -k 10 120 ./shim_bench 4 400 || exit $?
