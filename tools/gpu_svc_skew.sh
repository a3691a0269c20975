# Request-service latency per staged-block-stride skew (build/variants/s*.so,
# -DECW_SVC_SKEW), 4 KiB and 64 KiB calls, phase-traced.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
: > gpurun_out/svc_skew_$T.log
for v in s0 s256 s1k s2304 s0; do
echo "== $v" >> gpurun_out/svc_skew_$T.log
timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_skew_$T.log 2>&1 || { cat gpurun_out/svc_skew_$T.log; exit 1; }
LEN=65536 CALLS=2000 timeout -k 10 120 python tools/svc_latency.py build/variants/$v.so >> gpurun_out/svc_skew_$T.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/svc_skew_$T.log
