#!/bin/bash
# BASELINE config 3 (65,536 envs, full PPO iteration) in both dtypes and layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for ac in bf16 none; do for lay in nchw channels_last; do
  timeout -k 10 400 python tools/bench_ppo.py --envs ${ENVS:-65536} --update-steps 200 --autocast $ac --layout $lay > gpurun_out/c3_${ac}_${lay}.json 2> gpurun_out/c3_${ac}_${lay}.err || { tail -5 gpurun_out/c3_${ac}_${lay}.err; exit 1; }
  cat gpurun_out/c3_${ac}_${lay}.json
done; done
