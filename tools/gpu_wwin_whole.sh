# Write window on whole-block layouts the bench reports beside the tiled slab:
# split slab and pointer tables over separate allocations, window off vs on,
# interleaved in one process each.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/wwin_whole.log}
L=ecwide_amd/libecwide.so
: > $OUT
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 6 --chunk 67108864 --split --pad 0 $L@off $L@on 2>&1 | grep -v amdgpu >> $OUT || exit $?
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 6 --tables $L@off $L@on 2>&1 | grep -v amdgpu >> $OUT || exit $?
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 6 --tables $L@off $L@on 2>&1 | grep -v amdgpu >> $OUT || exit $?
