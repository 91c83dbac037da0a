#!/bin/bash
# GPU session: new PPO/train tests, then the config-3 PPO timing (fp32 and bf16).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-train}
timeout -k 10 900 python -m pytest tests/test_gpu_train.py tests/test_gpu_ppo_agent.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/bench_ppo.py --envs 65536 > gpurun_out/ppo_fp32_$TAG.json 2> gpurun_out/ppo_fp32_$TAG.err || { tail -30 gpurun_out/ppo_fp32_$TAG.err; exit 1; }
cat gpurun_out/ppo_fp32_$TAG.json
timeout -k 10 600 python tools/bench_ppo.py --envs 65536 --autocast bf16 > gpurun_out/ppo_bf16_$TAG.json 2> gpurun_out/ppo_bf16_$TAG.err || { tail -30 gpurun_out/ppo_bf16_$TAG.err; exit 1; }
cat gpurun_out/ppo_bf16_$TAG.json
exit $rc
