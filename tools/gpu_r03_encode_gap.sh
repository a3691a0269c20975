# Round 3: the tiled encode's gap to the math-free window microbenchmark
#  and the store-flavour / WRITE_SIZE question (item 7).
#  1. build/variants: base (nt sc0 sc1 stores, 2 launch windows), stnt (nt
#     stores), one (one launch, one tile per workgroup), stnt_one; each with
#     the write window off and on, interleaved on one allocation (tiled slab
#     geometry: 8 KiB pieces, parities in their own region)
#  2. build/storebench: store flavours, store-only and the encode's byte mix,
#     with and without the window; then WRITE_SIZE / FETCH_SIZE passes over it
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
V="build/variants/base.so build/variants/stnt.so build/variants/one.so build/variants/stnt_one.so"
AB=""
for v in $V; do AB="$AB $v@off $v@on"; done
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $AB 2>&1 | grep -v amdgpu > gpurun_out/r03_gap_ab.log || exit $?
cat gpurun_out/r03_gap_ab.log
timeout -k 10 120 build/storebench 5 > gpurun_out/r03_storebench.log 2>&1 || exit $?
timeout -k 10 120 build/storebench 5 0 >> gpurun_out/r03_storebench.log 2>&1 || exit $?
cat gpurun_out/r03_storebench.log
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_sb_w -o run -- $GRAFT_REPO_ROOT/build/storebench 1 > $GRAFT_REPO_ROOT/gpurun_out/r03_sb_w.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_sb_f -o run -- $GRAFT_REPO_ROOT/build/storebench 1 > $GRAFT_REPO_ROOT/gpurun_out/r03_sb_f.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python tools/pmc_kernels.py gpurun_out/r03_sb_w gpurun_out/r03_sb_f > gpurun_out/r03_storebench_pmc.log
cat gpurun_out/r03_storebench_pmc.log
cd /tmp
for v in base stnt; do
  P="python3 $GRAFT_REPO_ROOT/tools/kbench.py --stripes 8 --rounds 1 --iters 1 --chunk 8192 --split --pad 0 $GRAFT_REPO_ROOT/build/variants/$v.so"
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_enc_w_$v -o run -- $P > $GRAFT_REPO_ROOT/gpurun_out/r03_enc_w_$v.log 2>&1 || exit $?
done
cd $GRAFT_REPO_ROOT
for v in base stnt; do echo "== $v"; python tools/pmc_kernels.py gpurun_out/r03_enc_w_$v; done > gpurun_out/r03_encode_write_pmc.log
cat gpurun_out/r03_encode_write_pmc.log
