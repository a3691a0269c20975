# Write-window A/B (ECW_WRITE_WINDOW per launch, one build, one process per
# layout): block slab, tiled, whole-block split, single-stripe pointer mode;
# then the bench with the window forced off and with the default choice.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/wwin.log}
L=ecwide_amd/libecwide.so
V="$L@off $L@on $L@10,32 $L@12,128"
: > $OUT
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 3 --check $V 2>&1 | grep -v amdgpu >> $OUT || exit $?
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 3 --chunk 8192 --split --pad 0 $L@off $L@on 2>&1 | grep -v amdgpu >> $OUT || exit $?
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 3 --chunk 67108864 --split --pad 0 $L@off $L@on 2>&1 | grep -v amdgpu >> $OUT || exit $?
timeout -k 10 200 python tools/kbench.py --stripes 8 --rounds 3 --ptr $L@off $L@on 2>&1 | grep -v amdgpu >> $OUT || exit $?
ECW_WRITE_WINDOW=off timeout -k 10 300 python bench.py --cpu-seconds 0 2>&1 | grep -v amdgpu | tail -1 >> $OUT || exit $?
timeout -k 10 300 python bench.py --cpu-seconds 0 2>&1 | grep -v amdgpu | tail -1 >> $OUT || exit $?
