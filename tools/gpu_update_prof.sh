#!/bin/bash
# bf16 optimizer-step timing (tools/prof_update.py) under runtime settings RUNS ("A=1 B=2;;C=3"), REPS interleaved
# repeats, then one rocprofv3 kernel trace of the default settings with the per-kernel breakdown.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pu}; R=$GRAFT_REPO_ROOT
IFS=$'\n'
for r in $(seq 1 ${REPS:-2}); do
  i=0
  for e in $(echo "${RUNS:-X=0}" | sed 's/;;/\n/g'); do
    i=$((i+1))
    env $(echo $e | tr ' ' '\n') timeout -k 10 180 python tools/prof_update.py --batch 2048 --steps 200 ${PU_ARGS:-} > gpurun_out/${TAG}_r${i}_$r.json 2> gpurun_out/${TAG}_r${i}_$r.err || { tail -5 gpurun_out/${TAG}_r${i}_$r.err; exit 1; }
    echo "$e rep $r: $(tail -1 gpurun_out/${TAG}_r${i}_$r.json)"
  done
done
unset IFS
cd /tmp || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_kt" -o run --output-format csv -- python3 "$R/tools/prof_update.py" --batch 2048 --steps 50 ${PU_ARGS:-} > "$R/gpurun_out/${TAG}_kt.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_kt.log"; exit 1; }
python3 "$R/tools/prof_update.py" --summarize "$(find "$R/gpurun_out/${TAG}_kt" -name '*kernel_trace.csv' | sort | tail -1)" --steps 50 > "$R/gpurun_out/${TAG}_kernels.txt" 2>&1; head -30 "$R/gpurun_out/${TAG}_kernels.txt" | cut -c1-150
