# Round 3: SQ counters of the encode tiles (where the 5-8-row asm tile loses
# its time against the <=4-row one): RS(128, 3 / 5 / 8), 64 MiB blocks, two
# counter passes each, per-kernel means (tools/pmc_kernels.py).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
L=$GRAFT_REPO_ROOT/ecwide_amd/libecwide.so
P1=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_LDS_BANK_CONFLICT
P2=SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_WAVES,SQ_ACTIVE_INST_SCA,SQ_INSTS_SMEM,GRBM_GUI_ACTIVE,GRBM_COUNT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "more_than_8 or random_sweep" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pytest_m8.log 2>&1 || { tail -30 gpurun_out/r03_pytest_m8.log; exit 1; }
tail -1 gpurun_out/r03_pytest_m8.log
O=gpurun_out/r03_sq.log
: > $O
for m in 3 5 8; do
  A="python3 $GRAFT_REPO_ROOT/tools/kbench.py --code R --k 128 --m $m --stripes 4 --rounds 1 --iters 2 $L"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_sq1_m$m -o run -- $A > $GRAFT_REPO_ROOT/gpurun_out/r03_sq1_m$m.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r03_sq1_m$m.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $P2 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_sq2_m$m -o run -- $A > $GRAFT_REPO_ROOT/gpurun_out/r03_sq2_m$m.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/r03_sq2_m$m.log; exit 1; }
  cd $GRAFT_REPO_ROOT
  echo "== RS(128, $m)" >> $O
  grep "encode " gpurun_out/r03_sq1_m$m.log >> $O
  python tools/pmc_kernels.py gpurun_out/r03_sq1_m$m gpurun_out/r03_sq2_m$m | grep -v fill_ >> $O
done
cat $O
