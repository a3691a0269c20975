# block-stride padding sweep at the bench shape (k=128, 64 MiB, 8 stripes)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
: > gpurun_out/pad64.log
for pad in 4096 8192 12288 16384 24576 32768 65536 1052672 2101248; do
  echo "pad=$pad" >> gpurun_out/pad64.log
  timeout -k 10 200 python tools/kbench.py --mib 64 --stripes 8 --rounds 2 --iters 3 --pad $pad ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu | tail -1 >> gpurun_out/pad64.log || exit $?
done
