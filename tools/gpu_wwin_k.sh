# Write window: k around the auto threshold (96), the 5-8-row tile, RS.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/wwin_k2.log}
L=ecwide_amd/libecwide.so
V="$L@off $L@on"
: > $OUT
for A in "--k 64 --r 16 --m 3 --mib 64 --stripes 16" "--k 96 --r 24 --m 3 --mib 64 --stripes 8" "--k 128 --r 27 --m 3 --mib 64 --stripes 8" "--k 128 --r 27 --m 6 --mib 64 --stripes 8" "--k 128 --m 3 --mib 64 --stripes 8 --code R" "--k 128 --r 27 --m 3 --mib 64 --stripes 8 --ptr"; do
  timeout -k 10 200 python tools/kbench.py --rounds 3 $A $V 2>&1 | grep -v amdgpu >> $OUT || exit $?
done
