#!/usr/bin/env python3
"""CPU baselines of BASELINE.md §2 on this host's cores: ECWide-C's encodeData
+ decodeData flow (bench.cpu_baseline: the oracle's AVX2 port of ISA-L's
kernels, test infrastructure) at 1 thread (ECWide-C's one ComputeWorker) and
at the GPU's share of cores, on one whole stripe of each configuration, plus
the 4 MiB column sample the round-1 bench used, to show how it compares with
whole 64 MiB blocks. One JSON line per measurement."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402

CONFIGS = [
    ("configs[0] default scheme.ini CL(32,11,3)", 32, 3, 11, 64),
    ("configs[1] CL(k=32, 4 groups, m=2)", 32, 2, 8, 16),
    ("configs[2]/bench CL(128,27,3)", 128, 3, 27, 64),
    ("configs[2] shape, 4 MiB column sample (round-1 method)", 128, 3, 27, 4),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=bench.DEFAULT_SEED)
    a = ap.parse_args()
    for name, k, m, r, mib in CONFIGS:
        res = bench.cpu_baseline(a, k, m, r, mib << 20)
        print(json.dumps({"config": name, "k": k, "m": m, "r": r, "block_mib": mib, **res}), flush=True)


if __name__ == "__main__":
    main()
