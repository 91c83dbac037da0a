#!/bin/bash
# BASELINE config 3 end to end: run_train.py on 65,536 envs for 2 PPO updates
# (2 x (128 rollout steps + 40,960 minibatch steps)), bf16 autocast, on one MI355X.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
cd block-blast-ai---reinforcement-learning-agent_amd || exit 1
W=$(mktemp -d)
# an update takes minutes between log lines: keep gpurun_out/ moving
( while sleep 30; do date +%T >> "$GRAFT_REPO_ROOT/gpurun_out/train64k_heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
sed "s#checkpoints#$W/ck#; s#logs#$W/logs#; s#results#$W/res#; s#num_envs: 65536#num_envs: ${ENVS:-65536}#" config/${CFG:-gpu_64k_bf16}.yaml > $W/cfg.yaml
timeout -k 10 ${TL:-900} python -u run_train.py --config $W/cfg.yaml --max-updates ${UPD:-2} > "$GRAFT_REPO_ROOT/gpurun_out/train64k_${CFG:-gpu_64k_bf16}.log" 2>&1
rc=$?; tail -25 "$GRAFT_REPO_ROOT/gpurun_out/train64k_${CFG:-gpu_64k_bf16}.log"; exit $rc
