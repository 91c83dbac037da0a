#!/bin/bash
# SQ counters of the board-convolution kernels (tools/bench_conv.py, one shape),
# one rocprofv3 --pmc pass per counter set; prints per-dispatch averages.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-convpmc}
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
i=0
for set in ${SETS:-SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_INSTS_VALU,SQ_INSTS_LDS,SQ_INSTS_SALU,SQ_INSTS_VMEM,SQ_INSTS_MFMA}; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_$i" -o run --output-format csv -- python "$R/tools/bench_conv.py" --shapes ${SHAPE:-128x128} --reps 5 > "$R/gpurun_out/${TAG}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_$i.log"; echo "pass $i failed"; exit 1; }
done
python - "$R/gpurun_out" "$TAG" <<'PY'
import csv, glob, sys, collections, re
out, tag = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/{tag}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "bb::" not in k:
            continue
        m = re.search(r"namespace\)::(\w+(<[^>]*>)?)", k)
        name = m.group(1) if m else k[:60]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in acc.items():
    print(name, " ".join(f"{c}={sum(x)/len(x):.4g}" for c, x in sorted(cs.items())), "(per dispatch)")
PY
