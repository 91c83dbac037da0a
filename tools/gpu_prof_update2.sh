#!/bin/bash
# steady-state kernel breakdown of the bf16 update step, NCHW and channels_last
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for lay in nchw cl; do
  X=""; [ $lay = cl ] && X=--channels-last
  cd /tmp || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/pu_$lay" -o run --output-format csv -- python "$R/tools/prof_update.py" --autocast bf16 $X > "$R/gpurun_out/pu_$lay.log" 2>&1 || { tail -20 "$R/gpurun_out/pu_$lay.log"; exit 1; }
  cd "$R" || exit 1
  f=$(find "$R/gpurun_out/pu_$lay" -name "*kernel_trace.csv" | head -1)
  python tools/prof_update.py --summarize "$f" --steps 50 > gpurun_out/pu_${lay}.txt && head -45 gpurun_out/pu_${lay}.txt
  rm -rf "$R/gpurun_out/pu_$lay"
done
