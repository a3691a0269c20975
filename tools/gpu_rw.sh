# Read- vs write-layout A/B of the encode (tools/rw_layout.py).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r02}
timeout -k 10 300 python tools/rw_layout.py --rounds 3 --ptr-stripes 4 --alloc-stripes 4 > gpurun_out/rw_layout_$T.log 2>&1 || { cat gpurun_out/rw_layout_$T.log; exit 1; }
cat gpurun_out/rw_layout_$T.log
