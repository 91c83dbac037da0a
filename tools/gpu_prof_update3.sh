#!/bin/bash
# steady-state kernel breakdown of the bf16 update step (channels_last, the default layout)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; TAG=${1:-pu3}
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/$TAG" -o run --output-format csv -- python "$R/tools/prof_update.py" --autocast bf16 --channels-last > "$R/gpurun_out/$TAG.log" 2>&1 || { tail -20 "$R/gpurun_out/$TAG.log"; exit 1; }
cd "$R" || exit 1
f=$(find "$R/gpurun_out/$TAG" -name "*kernel_trace.csv" | head -1)
python tools/prof_update.py --summarize "$f" --steps 50 > gpurun_out/$TAG.txt && head -60 gpurun_out/$TAG.txt
rm -rf "$R/gpurun_out/$TAG"
