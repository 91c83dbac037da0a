#!/bin/bash
# update-step kernel breakdown for two library builds (tools/variants/libbbvec_<v>.so; main = in-tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-nnold main}; do
  lib=$R/tools/variants/libbbvec_$v.so; [ "$v" = main ] && lib=$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
  cd /tmp || exit 1
  BBVEC_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/pc_$v" -o run --output-format csv -- python "$R/tools/prof_update.py" --autocast bf16 --channels-last > "$R/gpurun_out/pc_$v.log" 2>&1 || { tail -20 "$R/gpurun_out/pc_$v.log"; exit 1; }
  cd "$R" || exit 1
  f=$(find "$R/gpurun_out/pc_$v" -name "*kernel_trace.csv" | head -1)
  python tools/prof_update.py --summarize "$f" --steps 50 > gpurun_out/pc_$v.txt || exit 1
  rm -rf "$R/gpurun_out/pc_$v"
  echo "== $v"; grep -E "marker|bn_" gpurun_out/pc_$v.txt | cut -c1-120
done
