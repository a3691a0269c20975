# block-stride padding sweep (default: the bench shape, k=128, 64 MiB, 8 stripes)
#   bash tools/gpu_pad.sh [MiB] [stripes]
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
MIB=${1:-64}; S=${2:-8}
: > gpurun_out/pad.log
for pad in 0 4096 8192 12288 16384 24576 32768 65536 69632 1052672 2101248; do
  echo "pad=$pad" >> gpurun_out/pad.log
  timeout -k 10 200 python tools/kbench.py --mib $MIB --stripes $S --rounds 2 --iters 3 --pad $pad ecwide_amd/libecwide.so 2>&1 | grep -v amdgpu | tail -1 >> gpurun_out/pad.log || exit $?
done
