#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_kernels.py tests/test_gpu_ppo_agent.py tests/test_gpu_train.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ppo.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_ppo.log
[ $rc -eq 0 ] || { grep -m3 -A30 "Error\|assert" gpurun_out/pytest_ppo.log | head -60; exit $rc; }
for v in ${VARS:-"bf16:--autocast bf16 --no-graph" "fp32:--no-graph"}; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 400 python tools/bench_ppo.py --envs ${ENVS:-8192} --update-steps 200 $a > gpurun_out/ppog_$n.json 2> gpurun_out/ppog_$n.err || { tail -5 gpurun_out/ppog_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ppog_$n.json'));print('$n', d['update_step_ms'], d['update_cnn_tflops'], d['rollout_env_steps_per_s'])"
done
