#!/usr/bin/env python3
"""Diagnostics (not product): per-launch averages of the PMC counters of one kernel from rocprofv3
--pmc passes (tools/gpu_sq_async.sh).  usage: sq_summary.py OUT_DIR TAG KERNEL_SUBSTRING [--json FILE
--envs N --steps-per-launch T]: with --json, also the instruction-issue record bench.py puts in its
line as roofline.valu (profiles/sq_rollout_kernel.json)."""
import collections
import csv
import glob
import json
import sys

SIMDS = 1024  # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)
XCDS = 8  # GRBM_GUI_ACTIVE sums the GPU-busy cycles of the 8 XCDs
# measured VALU issue floor with two waves per SIMD (profiles/r04/sqa1_valu_rates.txt, tools/ubench): one
# wave-instruction per 2.9 cycles (v_add_u32, 5.79 / 2) to 3.7 cycles (64-bit shifts, 7.41 / 2) per SIMD
FLOOR_CYCLES = (2.9, 3.7)


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
    mean = {}
    for c, v in sorted(acc.items()):
        # warm-up launches included: report the mean of the last half (steady state)
        tail = v[len(v) // 2:]
        mean[c] = sum(tail) / len(tail)
        print(f"{c:28s} {mean[c]:18.1f}  per launch (n={len(tail)})")
    if "--json" in sys.argv:
        arg = lambda k, d: type(d)(sys.argv[sys.argv.index(k) + 1]) if k in sys.argv else d
        n, t = arg("--envs", 65536), arg("--steps-per-launch", 128)
        es = n * t
        valu, wc, gui = mean.get("SQ_INSTS_VALU"), mean.get("SQ_WAVE_CYCLES"), mean.get("GRBM_GUI_ACTIVE")
        rec = {"kernel": kern, "n_envs": n, "steps_per_launch": t, "counters_per_launch": mean,
               "profiled_ms": round(sum(dur) / len(dur), 5) if dur else None}
        if valu:
            rec["valu_insts_per_launch"] = round(valu)
            rec["valu_insts_per_env_step"] = round(valu / es, 2)
        if wc:
            rec["wave_cycles_per_env_step"] = round(wc / es, 2)
        if valu and gui:
            cyc = gui / XCDS  # busy cycles of one XCD over the launch
            per = cyc * SIMDS / valu  # cycles between VALU issues of one SIMD
            rec["cycles_per_valu_per_simd"] = round(per, 3)
            rec["issue_floor_cycles"] = list(FLOOR_CYCLES)
            rec["issue_frac"] = [round(FLOOR_CYCLES[0] / per, 3), round(FLOOR_CYCLES[1] / per, 3)]
        try:  # the sources the profiled library was built from (runtime.lib.load() refuses any other)
            import os
            sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "block-blast-ai---reinforcement-learning-agent_amd"))
            from runtime.build import source_id
            rec["build_id"] = source_id()
        except Exception:  # noqa: BLE001
            pass
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
