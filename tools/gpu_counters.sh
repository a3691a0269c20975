# SQ-level counters for the encode kernel (each --pmc pass separately; no
# trace domains combined with --pmc).
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
cd /tmp
P="python3 $GRAFT_REPO_ROOT/tools/kbench.py --stripes 2 --rounds 1 --iters 2 $GRAFT_REPO_ROOT/ecwide_amd/libecwide.so"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sq1 -o run -- $P > $GRAFT_REPO_ROOT/gpurun_out/sq1.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sq2 -o run -- $P > $GRAFT_REPO_ROOT/gpurun_out/sq2.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/sq3 -o run -- $P > $GRAFT_REPO_ROOT/gpurun_out/sq3.log 2>&1 || echo "sq3 pass failed (counter names)"
echo counters done
