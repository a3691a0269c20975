# Round 3: VALU / LDS issue rates of the encode tile's instruction mix
# (tools/csrc/valubench.hip, build/valubench built in-tree beforehand).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 build/valubench 20000 > gpurun_out/r03_valubench.log 2>&1 || { cat gpurun_out/r03_valubench.log; exit 1; }
cat gpurun_out/r03_valubench.log
