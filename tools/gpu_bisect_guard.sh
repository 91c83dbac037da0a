#!/bin/bash
# Diagnostics: which earlier GPU test files make test_train_checkpoints_logs_and_resume trip the Adam guard.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=tests/test_gpu_train.py::test_train_checkpoints_logs_and_resume
G1="tests/test_gpu_linear_tail.py tests/test_gpu_network_oracle.py"
G2="tests/test_gpu_optim.py"
G3="tests/test_gpu_ppo_agent.py"
G4="tests/test_gpu_ppo_kernels.py tests/test_gpu_ppo_update_oracle.py"
G5="tests/test_gpu_rollout.py tests/test_gpu_single_env.py tests/test_gpu_solver_stress.py"
for g in ${GROUPS_:-G1 G2 G3 G4 G5}; do
  eval files=\$$g
  timeout -k 10 500 python -u -m pytest $files $T -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/bis_$g.log 2>&1
  echo "$g rc=$? $(tail -1 gpurun_out/bis_$g.log) guard_lines=$(grep -c 'guard:' gpurun_out/bis_$g.log)"
done
