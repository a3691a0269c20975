# Round 3: tiny encodes through every path with each launch synchronised,
# then (only if they pass) the GPU suite.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ECW_DEBUG_LAUNCH=1 ECW_SERVICE=0 timeout -k 10 60 python tools/dbg_encode.py ecwide_amd/libecwide.so > gpurun_out/r03_dbg.log 2>&1 || { cat gpurun_out/r03_dbg.log; exit 1; }
timeout -k 10 60 python tools/dbg_encode.py ecwide_amd/libecwide.so >> gpurun_out/r03_dbg.log 2>&1 || { cat gpurun_out/r03_dbg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_dbg.log | tail -12
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r03_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03_pytest_gpu.log
