#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ppo2}
for args in "" "--miopen-find" "--channels-last" "--miopen-find --channels-last" "--autocast bf16 --miopen-find"; do
  timeout -k 10 400 python tools/bench_ppo.py --envs 65536 --update-steps 60 $args > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}.json'));print('$args', d['rollout_s'], d['update_step_ms'], d['ppo_env_steps_per_s'])"
done
