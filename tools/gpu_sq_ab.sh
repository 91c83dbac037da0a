#!/bin/bash
# SQ instruction counters of bb::rollout_kernel per library variant (tools/variants.py),
# one --pmc pass per counter set:  VARIANTS="main diag1" bash tools/gpu_sq_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sqab}
R=$GRAFT_REPO_ROOT
cd /tmp || exit 1
for v in ${VARIANTS:-main}; do
  i=0
  for set in ${SETS:-SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_BRANCH}; do
    i=$((i+1))
    lib=$R/tools/variants/libbbvec_$v.so; [ "$v" = main ] && lib=$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
    BBVEC_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc ${set//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_$i" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 10 --warmup 5 > "$R/gpurun_out/${TAG}_${v}_$i.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${v}_$i.log"; echo "pass $v $i failed"; exit 1; }
  done
done
python - "$R/gpurun_out" "$TAG" ${VARIANTS:-main} <<'PY'
import csv, glob, sys, collections
out, tag, vs = sys.argv[1], sys.argv[2], sys.argv[3:]
for v in vs:
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{out}/{tag}_{v}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "bb::rollout" in r.get("Kernel_Name", ""):  # rollout_kernel / rollout_async_kernel
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    ws = 2048 * 128  # wave-steps per launch (65,536 envs / 32 per wave, T = 128): counters per 32 env-steps
    print(v, " ".join(f"{c}={sum(x)/len(x)/ws:.1f}" for c, x in sorted(acc.items()) if c != "SQ_WAVES"), "(per wave-step)")
PY
