# Tiled slab, write window off / on with the launch-window schedule, the
# ticket-ordered schedule (tables staged once per workgroup) and without the
# table staging (timing only) -- is the window's loss on the tiled slab the
# per-generation staging bubble?
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/wwin_ticket.log}
V=""
for n in base ticket nostage; do for e in off on 12,128; do V="$V build/variants/$n.so@$e"; done; done
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 4 --chunk 8192 --split --pad 0 $V 2>&1 | grep -v amdgpu > $OUT || exit $?
cat $OUT
