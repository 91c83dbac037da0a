#!/usr/bin/env python3
"""Diagnostics (not product): per-launch averages of the PMC counters of one kernel from rocprofv3
--pmc passes (tools/gpu_sq_async.sh).  usage: sq_summary.py OUT_DIR TAG KERNEL_SUBSTRING"""
import collections
import csv
import glob
import sys


def main():
    out, tag, kern = sys.argv[1], sys.argv[2], sys.argv[3]
    acc = collections.defaultdict(list)
    dur = []
    for f in glob.glob(f"{out}/{tag}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r.get("Kernel_Name", ""):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in glob.glob(f"{out}/{tag}_p*/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kern in r.get("Kernel_Name", ""):
                dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    if dur:
        print(f"{kern}: {len(dur)} launches, mean duration {sum(dur) / len(dur):.4f} ms (under the profiler)")
    for c, v in sorted(acc.items()):
        # warm-up launches included: report the mean of the last half (steady state)
        tail = v[len(v) // 2:]
        print(f"{c:28s} {sum(tail) / len(tail):18.1f}  per launch (n={len(tail)})")


if __name__ == "__main__":
    main()
