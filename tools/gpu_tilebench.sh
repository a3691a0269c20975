# tools/csrc/tilebench.hip: the encode's byte mix with XOR for math, tile widths and output layouts.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
hipcc --offload-arch=gfx950 -O3 tools/csrc/tilebench.hip -o /tmp/tilebench || exit 1
timeout -k 10 300 /tmp/tilebench 5 > gpurun_out/tilebench_$T.log 2>&1 || { cat gpurun_out/tilebench_$T.log; exit 1; }
cat gpurun_out/tilebench_$T.log
