# Request-service variants (build/variants/p*u*.so: parts per slot x column
# unit): 4 KiB and 64 KiB single-thread latency, 4 and 16 threads.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
: > gpurun_out/svc_units_$T.log
for v in ${VARIANTS:-p8u1k p8u256 p16u256 p16u512 p32u256 p8u1k}; do
echo "== $v" >> gpurun_out/svc_units_$T.log
timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_units_$T.log 2>&1 || { cat gpurun_out/svc_units_$T.log; exit 1; }
LEN=65536 CALLS=2000 timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_units_$T.log 2>&1 || exit $?
THREADS=4 CALLS=2000 timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_units_$T.log 2>&1 || exit $?
THREADS=16 CALLS=1000 timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_units_$T.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/svc_units_$T.log
