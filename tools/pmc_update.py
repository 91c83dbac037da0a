#!/usr/bin/env python3
"""Diagnostics: HBM bytes per dispatch of every kernel of the bf16 update step, from two rocprofv3 PMC passes
over tools/prof_update.py (FETCH_SIZE doubled for gfx950 and WRITE_SIZE, MI355X_MICROARCH.md §HBM), beside the
mean duration from a plain kernel trace of the same command: achieved HBM GB/s per kernel.

    python tools/pmc_update.py KT_DIR FETCH_DIR WRITE_DIR [--out FILE]
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def _short(name: str) -> str:
    name = name.replace("bb::(anonymous namespace)::", "")
    return name.split("(")[0][:70]


def _rows(d: str, pattern: str):
    files = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    if not files:
        raise SystemExit(f"no {pattern} under {d}")
    for f in files:
        with open(f) as fh:
            yield from csv.DictReader(fh)


def counters(d: str, counter: str):
    acc = defaultdict(list)
    for r in _rows(d, "*counter_collection.csv"):
        if r.get("Counter_Name") == counter:
            acc[_short(r.get("Kernel_Name", ""))].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def durations(d: str):
    acc = defaultdict(list)
    for r in _rows(d, "*kernel_trace.csv"):
        acc[_short(r.get("Kernel_Name", ""))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kt_dir")
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    fetch, write, dur = counters(a.fetch_dir, "FETCH_SIZE"), counters(a.write_dir, "WRITE_SIZE"), durations(a.kt_dir)
    lines = [f"{'kernel':70s} {'calls':>6s} {'us':>7s} {'read MB':>8s} {'write MB':>8s} {'GB/s':>7s}"]
    rows = []
    for k, (t, n) in dur.items():
        rd, wr = 2 * fetch.get(k, 0.0), write.get(k, 0.0)
        rows.append((t * n, k, n, t, rd, wr))
    for _, k, n, t, rd, wr in sorted(rows, reverse=True):
        lines.append(f"{k:70s} {n:6d} {t * 1e6:7.1f} {rd / 1e6:8.2f} {wr / 1e6:8.2f} {(rd + wr) / t / 1e9:7.0f}")
    s = "\n".join(lines)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
