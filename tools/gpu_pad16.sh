cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/pad16.log
for pad in 0 4096 8192 12288 69632 266240 1060864; do
  echo "pad=$pad" >> gpurun_out/pad16.log
  timeout -k 10 200 python tools/kbench.py --mib 16 --stripes 32 --rounds 2 --iters 3 --pad $pad ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu | tail -1 >> gpurun_out/pad16.log || exit $?
done
for pad in 0 4096 69632; do
  echo "B=64MiB pad=$pad" >> gpurun_out/pad16.log
  timeout -k 10 200 python tools/kbench.py --mib 64 --stripes 8 --rounds 2 --iters 3 --pad $pad ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu | tail -1 >> gpurun_out/pad16.log || exit $?
done
