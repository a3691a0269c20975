# Placement study, translation side: UTCL2 busy cycles per encode dispatch
# next to the per-slab rates of the same process.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pl2 && export TMPDIR=/tmp
i=0
for C in "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/pl2/p$i -o run --output-format csv -- python3 tools/placement_pmc.py --rounds 4 > gpurun_out/pl2/p$i.log 2>&1 || { tail -20 gpurun_out/pl2/p$i.log; exit 1; }
  grep "^slab" gpurun_out/pl2/p$i.log
  f=$(find gpurun_out/pl2/p$i -name '*counter_collection.csv' | head -1)
  python tools/placement_pmc.py --summarize $f --rounds 4
done
