#!/usr/bin/env python3
"""HBM traffic per bb_step / bb_rollout launch from two rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT/fetch ... -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d OUT/write ... -- python bench.py ...
    python tools/pmc_traffic.py OUT/fetch OUT/write --envs 65536 --out FILE

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  Per MI355X_MICROARCH.md
(§HBM): on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads,
so it is doubled; WRITE_SIZE is taken as is.  The per-launch figure is the
mean over dispatches of each bb_step kernel, summed over the two kernels of
one bb_step (step_fused_kernel, or step_kernel + escalate_kernel), or the rollout_async_kernel of a
bb_rollout launch (--kernels rollout_async_kernel --steps-per-launch T).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

def per_kernel(d: str, counter: str, KERNELS):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                for k in KERNELS:
                    if f"bb::{k}(" in name or f"bb::{k}<" in name:
                        acc[k].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items() if v}, {k: len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--out", default=None)
    ap.add_argument("--kernels", default="step_kernel,escalate_kernel")
    ap.add_argument("--steps-per-launch", type=int, default=1)
    a = ap.parse_args()
    KERNELS = tuple(a.kernels.split(","))
    fetch, nf = per_kernel(a.fetch_dir, "FETCH_SIZE", KERNELS)
    write, nw = per_kernel(a.write_dir, "WRITE_SIZE", KERNELS)
    kib = 1024.0
    per = {k: {"fetch_bytes_x2": 2 * fetch.get(k, 0.0) * kib, "write_bytes": write.get(k, 0.0) * kib,
               "dispatches": [nf.get(k, 0), nw.get(k, 0)]} for k in KERNELS}
    total = sum(v["fetch_bytes_x2"] + v["write_bytes"] for v in per.values())
    out = {"n_envs": a.envs, "steps_per_launch": a.steps_per_launch, "hbm_bytes_per_launch": round(total),
           "per_kernel": per, "bytes_per_env_step": round(total / a.envs / a.steps_per_launch, 2),
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes; FETCH_SIZE x2 (gfx950)"}
    try:  # the sources the profiled library was built from (runtime.lib.load() refuses any other)
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "block-blast-ai---reinforcement-learning-agent_amd"))
        from runtime.build import source_id
        out["build_id"] = source_id()
    except Exception:  # noqa: BLE001
        pass
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
