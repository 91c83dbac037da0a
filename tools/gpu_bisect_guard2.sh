#!/bin/bash
# Diagnostics: which code path of tests/test_gpu_ppo_agent.py makes the later train() trip the Adam guard.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=tests/test_gpu_train.py::test_train_checkpoints_logs_and_resume
P=tests/test_gpu_ppo_agent.py
run() {  # name, env, pytest -k filter for the agent tests
  env $2 timeout -k 10 300 python -u -m pytest $P $T -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "$3" > gpurun_out/bis2_$1.log 2>&1
  echo "$1 [$2] [$3] rc=$? $(tail -1 gpurun_out/bis2_$1.log) guard=$(grep -c 'guard:' gpurun_out/bis2_$1.log)"
}
run base "X=0" "test_"
run nopig "BB_WGRAD_PIGGYBACK=0" "test_"
run notail "BB_LINEAR_TAIL=0" "test_"
run nohipconv "BB_HIP_CONV=0" "test_"
run nof32conv "BB_F32_CONV=0" "test_"
run nostats "BB_CONV_STATS=0" "test_"
run g32 "X=0" "train_checkpoints or (graphed and None)"
run gbf "X=0" "train_checkpoints or (graphed and bfloat16)"
run other "X=0" "not graphed"
