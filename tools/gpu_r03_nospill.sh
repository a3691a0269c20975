# Round 3: the spill-free encode (r03.so) against round 2's build (base.so):
# interleaved A/B on one allocation per layout, the FETCH/WRITE_SIZE passes of
# the new tiled encode, then the default bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
O=gpurun_out/r03_nospill_ab.log
B=build/variants/base.so; N=build/variants/r03.so
echo "== tiled (8 KiB pieces, parities apart)" > $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --chunk 8192 --split --pad 0 $B $N $B@on $N@on 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== block slab (window on by default)" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --check $B $N $N@off 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== pointer tables over separate allocations" >> $O
timeout -k 10 300 python tools/kbench.py --stripes 8 --rounds 5 --tables $B $N $N@off 2>&1 | grep -v amdgpu >> $O || exit $?
echo "== k=32 r=8 m=2 16 MiB x32 (configs[1] shape), block slab" >> $O
timeout -k 10 300 python tools/kbench.py --k 32 --r 8 --m 2 --mib 16 --stripes 32 --rounds 5 $B $N 2>&1 | grep -v amdgpu >> $O || exit $?
cat $O
cd /tmp
P="python3 $GRAFT_REPO_ROOT/tools/kbench.py --stripes 8 --rounds 1 --iters 1 --chunk 8192 --split --pad 0 $GRAFT_REPO_ROOT/$N"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_enc_w_new -o run -- $P > $GRAFT_REPO_ROOT/gpurun_out/r03_enc_w_new.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03_enc_f_new -o run -- $P > $GRAFT_REPO_ROOT/gpurun_out/r03_enc_f_new.log 2>&1 || exit $?
cd $GRAFT_REPO_ROOT
python tools/pmc_kernels.py gpurun_out/r03_enc_w_new gpurun_out/r03_enc_f_new | tee gpurun_out/r03_encode_pmc_new.log
timeout -k 10 600 python bench.py > gpurun_out/r03_bench_first.log 2>&1 || { tail -30 gpurun_out/r03_bench_first.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_bench_first.log | tail -3
