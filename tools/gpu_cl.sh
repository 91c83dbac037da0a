#!/bin/bash
# PPO-update kernels + agent tests, then the update step's steady state in both layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_kernels.py tests/test_gpu_ppo_agent.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_cl.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_cl.log; [ $rc -eq 0 ] || { grep -m2 -B5 -A30 "Error\|assert" gpurun_out/pytest_cl.log | head -80; exit $rc; }
for a in "--autocast bf16" "--autocast bf16 --channels-last" "--autocast none" "--autocast none --channels-last"; do
  timeout -k 10 200 python tools/prof_update.py $a 2>/dev/null || exit 1
done
ACS="bf16" EXTRA=--channels-last bash tools/gpu_prof_update.sh 2>/dev/null
