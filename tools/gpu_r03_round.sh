# Round 3 end-to-end check on one box: the GPU suite, smoke, the default bench,
# configs[3], the N=2 self-launch, then the driver's torchrun form at N=2 / 4.
cd $GRAFT_REPO_ROOT && bash tools/gpu_check.sh && bash tools/gpu_ranks.sh
