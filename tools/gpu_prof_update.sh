#!/bin/bash
# steady-state kernel breakdown of the config-3 optimizer step (tools/prof_update.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for ac in ${ACS:-bf16 none}; do
  timeout -k 10 300 python tools/prof_update.py --autocast $ac $EXTRA || exit 1
  cd /tmp || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/pu_$ac" -o run --output-format csv -- python "$R/tools/prof_update.py" --autocast $ac $EXTRA > "$R/gpurun_out/pu_$ac.log" 2>&1 || { tail -20 "$R/gpurun_out/pu_$ac.log"; exit 1; }
  cd "$R" || exit 1
  f=$(find "$R/gpurun_out/pu_$ac" -name "*kernel_trace.csv" | head -1)
  python tools/prof_update.py --summarize "$f" --steps 50 > gpurun_out/pu_${ac}.txt && cat gpurun_out/pu_${ac}.txt
  rm -rf "$R/gpurun_out/pu_$ac"
done
