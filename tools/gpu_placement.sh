# Placement study (tools/placement_pmc.py): rates of 4 identical slabs in one
# process, then the same under PMC passes (one counter set per pass).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/pl && export TMPDIR=/tmp
timeout -k 10 200 python tools/placement_pmc.py > gpurun_out/pl/rates.log 2>&1 || { tail -20 gpurun_out/pl/rates.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pl/rates.log
i=0
for C in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum" "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum" "TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $C -d gpurun_out/pl/p$i -o run --output-format csv -- python3 tools/placement_pmc.py > gpurun_out/pl/p$i.log 2>&1 || { tail -20 gpurun_out/pl/p$i.log; exit 1; }
  grep "^slab" gpurun_out/pl/p$i.log
  f=$(find gpurun_out/pl/p$i -name '*counter_collection.csv' | head -1)
  python tools/placement_pmc.py --summarize $f
done
