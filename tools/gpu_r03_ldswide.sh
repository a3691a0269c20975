# Round 3: LDS issue rate of wide nibble lookups (ds_read_b64 / b96 / b128)
# against ds_read_b32 (tools/csrc/valubench.hip mode 1; build/valubench built in-tree).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 build/valubench 20000 1 > gpurun_out/r03_lds_wide.log 2>&1 || { cat gpurun_out/r03_lds_wide.log; exit 1; }
cat gpurun_out/r03_lds_wide.log
