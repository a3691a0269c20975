# Prototype: bit-sliced encode (tools/csrc/bitslice.hip, 4 KiB tiles) against
# the product's 5-8-row and 9-16-row LDS tiles, bench geometry, parity first.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
O=gpurun_out/bitslice_m_ab.log
: > $O
for args in "--code R --m 5" "--code R --m 8" "--code R --m 12" "--code R --m 16" "--m 10 --r 27" "--code R --m 3"; do
  echo "== $args" >> $O
  timeout -k 10 300 python tools/bitslice_ab.py $args --stripes 4 --rounds 3 build/bs_m.so 2>&1 | grep -v amdgpu >> $O || { cat $O; exit 1; }
done
cat $O
