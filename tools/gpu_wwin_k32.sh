# Write window at the k = 32 BASELINE shapes (block slab, pointer mode) and
# small k, where a tile's reads take a few windows' time.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/wwin_k32.log}
L=ecwide_amd/libecwide.so
V="$L@off $L@on $L@10,32 $L@12,128"
: > $OUT
for A in "--k 32 --r 11 --m 3 --mib 64 --stripes 8" "--k 32 --r 8 --m 2 --mib 16 --stripes 32" "--k 32 --r 11 --m 3 --mib 64 --stripes 8 --ptr" "--k 8 --r 4 --m 2 --mib 64 --stripes 32" "--k 200 --r 40 --m 4 --mib 16 --stripes 8"; do
  timeout -k 10 200 python tools/kbench.py --rounds 3 $A $V 2>&1 | grep -v amdgpu >> $OUT || exit $?
done
