# Phase latency of the request service (tools/svc_latency.py) for builds with 1/2/4/8 parts per slot.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
for v in p4 p8 p16; do
timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_trace_$T.log 2>&1 || { cat gpurun_out/svc_trace_$T.log; exit 1; }
LEN=65536 CALLS=2000 timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_trace_$T.log 2>&1 || exit $?
done
cat gpurun_out/svc_trace_$T.log
