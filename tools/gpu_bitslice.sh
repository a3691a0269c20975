# Prototype: bit-sliced encode tile vs the product encode on the bench's tiled
# geometry (k=128, 8 x 64 MiB as 8 KiB units), parity checked first.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/bitslice_ab.log
: > $O
for args in "${@:-}"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/bitslice_ab.py $args ${BS_LIBS:-build/bs_t5.so build/bs_t5d1.so build/bs_t5d2.so build/bs_t5nq.so build/bs_abl128.so} 2>&1 | grep -v amdgpu >> $O || { cat $O; exit 1; }
done
cat $O
