#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 --pmc counters (tools only).

  python tools/pmc_kernels.py DIR [DIR ...]

Finds every *counter_collection.csv under the given rocprofv3 output
directories and prints, per kernel name and counter, the number of
dispatches and the mean value per dispatch. FETCH_SIZE / WRITE_SIZE are KiB
per dispatch; the bytes column applies the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE x2 for 16 B/lane streams).
"""
import collections
import csv
import glob
import os
import sys


def main(dirs):
    acc = collections.defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    acc[(r.get("Kernel_Name", "?"), r.get("Counter_Name", "?"))].append(float(r["Counter_Value"]))
    for (kern, ctr), vals in sorted(acc.items()):
        mean = sum(vals) / len(vals)
        extra = ""
        if ctr == "WRITE_SIZE":
            extra = f"  = {mean * 1024 / 1e9:.4f} GB"
        elif ctr == "FETCH_SIZE":
            extra = f"  = {mean * 2048 / 1e9:.4f} GB (x2)"
        print(f"{ctr:12s} x{len(vals):3d} mean {mean:16.1f}{extra}  {kern[:120]}")


if __name__ == "__main__":
    main(sys.argv[1:])
