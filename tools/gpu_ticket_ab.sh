# ticket-ordered single launch (-DECW_TICKET=1) vs launch windows: parity check
# against the default build, then the same-allocation A/B at two slab sizes
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
V=build/variants
timeout -k 10 300 python -u tools/kbench.py --check --stripes 4 --rounds 2 --iters 2 $V/base.so $V/ticket.so > gpurun_out/ticket_check.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ticket_check.log
LIBS="base ticket" bash tools/gpu_grid_ab.sh
