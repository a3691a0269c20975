# Request service: parts per slot (build/variants/p4.so, p8.so) through the
# C shim callers; each variant is copied over the box's libecwide.so in turn.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
cd tools/csrc && gcc -O2 -o /tmp/shim_bench shim_bench.c -L../../ecwide_amd -lecw_isal -lpthread -Wl,-rpath,$GRAFT_REPO_ROOT/ecwide_amd || exit 1
cd $GRAFT_REPO_ROOT
: > gpurun_out/svc_parts_$T.log
for v in ${VARIANTS:-p8 p4 p8 p4}; do
  cp build/variants/$v.so ecwide_amd/libecwide.so || exit 1
  echo "== $v" >> gpurun_out/svc_parts_$T.log
  for t in 1 4 16; do timeout -k 10 120 /tmp/shim_bench $t 2000 >> gpurun_out/svc_parts_$T.log 2>&1 || exit $?; done
  timeout -k 10 120 /tmp/shim_bench 4 1000 seq >> gpurun_out/svc_parts_$T.log 2>&1 || exit $?
  LEN=65536 CALLS=1000 timeout -k 10 120 python tools/svc_latency.py ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu.ids >> gpurun_out/svc_parts_$T.log || exit 1
done
cat gpurun_out/svc_parts_$T.log
