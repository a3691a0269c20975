# 8 MiB blocks: encode + repair rate against the slab size (8 .. 256 stripes = 8.5 .. 272 GiB)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
B="python -u bench.py --block-mib 8 --cpu-seconds 0 --other-layout-steps 0 --steps 10 --warmup 2"
for S in 8 32 64 128 256; do
  timeout -k 10 300 $B --stripes $S > gpurun_out/sz_$S.log 2>&1 || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/sz_$S.log').read().strip().splitlines()[-1]);print($S, d['value'], d['encode_GBps'], d['repair_GBps'])"
done
