#!/usr/bin/env python3
"""Summarise rocprofv3 output into profiles/.

  kernel stats : python tools/prof_summary.py stats <run_results.db|kernel_stats.csv> <out.csv>
  PMC traffic  : python tools/prof_summary.py pmc <fetch counter_collection.csv> <write counter_collection.csv>
                 <kernel-substring> <algorithmic bytes per launch> <out.json> <config-key>

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reads
exactly 1/2 of the bytes of a wide (16 B/lane) coalesced streaming read
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores.
"""
import csv
import json
import os
import sqlite3
import sys


def stats(src, out):
    rows = []
    if src.endswith(".db"):
        c = sqlite3.connect(src)
        # the rocpd top_kernels view reports microseconds; store ns like the CSV output
        for name, calls, total, avg, pct in c.execute("select * from top_kernels"):
            rows.append([name, calls, total * 1e3, avg * 1e3, pct])
    else:
        with open(src) as f:
            for r in csv.DictReader(f):
                rows.append([r["Name"], r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["Percentage"]])
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        w.writerows(rows)
    for r in rows:
        print(f"{float(r[3]) / 1e6:10.4f} ms avg  x{r[1]:>4}  {r[0][:110]}")


def _per_dispatch(path, counter, needle):
    vals = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if needle in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                vals.append(float(r["Counter_Value"]))
    return vals


def pmc(fetch_csv, write_csv, needle, alg_bytes, out_json, key):
    fe = _per_dispatch(fetch_csv, "FETCH_SIZE", needle)
    wr = _per_dispatch(write_csv, "WRITE_SIZE", needle)
    if not fe or not wr:
        raise SystemExit(f"no {needle} dispatches with FETCH_SIZE/WRITE_SIZE")
    fetch = sum(fe) / len(fe) * 1024 * 2  # gfx950: FETCH_SIZE = 1/2 of streamed bytes
    write = sum(wr) / len(wr) * 1024
    d = json.load(open(out_json)) if os.path.exists(out_json) else {}
    d[key] = {
        "kernel": needle,
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "encode_hbm_bytes_per_launch": fetch + write,
        "algorithmic_bytes_per_launch": float(alg_bytes),
        "traffic_over_algorithmic": (fetch + write) / float(alg_bytes),
        "dispatches": [len(fe), len(wr)],
        "correction": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16B/lane streams); WRITE_SIZE KiB x1024",
    }
    json.dump(d, open(out_json, "w"), indent=1, sort_keys=True)
    print(json.dumps(d[key], indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    else:
        pmc(*sys.argv[2:8])
