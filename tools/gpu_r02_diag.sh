#!/bin/bash
# Round-2 rollout diagnostics: phase cycles (diag3 build, tools/diag_rollout.py)
# and SQ instruction / wait counters of bb::rollout_kernel (separate --pmc passes).
#   variants built beforehand: python tools/variants.py build diag3
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r02d}
V=diag3 bash tools/gpu_diag_roll.sh || exit 1
cp gpurun_out/diag_roll_diag3.json gpurun_out/${TAG}_diag_roll.json
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
i=0
for set in SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY \
           SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_INST_CYCLES_SALU,SQ_WAIT_INST_LDS,SQ_BUSY_CYCLES,SQ_INSTS_BRANCH,SQ_INSTS_VMEM_WR; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_sq$i" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 5 > "$R/gpurun_out/${TAG}_sq$i.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_sq$i.log"; echo "pass $i failed"; exit 1; }
done
python - "$R/gpurun_out" "$TAG" <<'PY'
import csv, glob, sys, collections
out, tag = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(f"{out}/{tag}_sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "bb::rollout_kernel" in r.get("Kernel_Name", ""):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(acc.items()):
    print(f"{c:22s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
