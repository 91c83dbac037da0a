#!/bin/bash
# The fp32 optimizer step (config 3's precision) with the GEMV bias gradients against F.linear's, interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2 3; do
  for g in 1 0; do
    BB_F32_LINEAR_GEMV=$g timeout -k 10 180 python tools/prof_update.py --autocast none --batch 2048 --steps 100 > gpurun_out/f32s_${g}_$r.json 2> gpurun_out/f32s_${g}_$r.err || { tail -5 gpurun_out/f32s_${g}_$r.err; exit 1; }
    echo "gemv=$g $r $(cat gpurun_out/f32s_${g}_$r.json)"
  done
done
