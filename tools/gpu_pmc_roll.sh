#!/bin/bash
# SQ counters of bb::rollout_kernel at the bench shape, one rocprofv3 --pmc
# pass per counter set (kernel trace only), summarised per launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sqr}
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters.txt" 2>&1 || true
i=0
for set in ${SETS:-SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_SCA,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES,SQ_INSTS_BRANCH,SQ_ACTIVE_INST_MISC,SQ_INSTS_SMEM}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_$i" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline ${ARGS:---steps 10 --warmup 3} > "$R/gpurun_out/${TAG}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_$i.log"; echo "pass $i failed"; exit 1; }
done
python - "$R/gpurun_out" "$TAG" <<'PY'
import csv, glob, sys, collections
out, tag = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(f"{out}/{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        for kn in ("step_kernel", "escalate_kernel", "rollout_kernel"):
            if f"bb::{kn}(" in k or f"bb::{kn}<" in k:
                acc[(kn, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (kn, c), v in sorted(acc.items()):
    print(f"{kn:16s} {c:22s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
