#!/bin/bash
# Early exit of the exact phase: parity (env, solver stress, full size), rollout and step A/B vs the previous
# build, the T = 1 tail diagnostics.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-exit}
timeout -k 10 700 python -u -m pytest tests/test_gpu_solver_stress.py tests/test_gpu_full_parity.py tests/test_gpu_env_parity.py tests/test_gpu_single_env.py tests/test_gpu_rollout.py tests/test_gpu_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="${RV:-prev main}" PARITY=0 REPS=3 ARGS="--steps 640 --warmup 64" bash tools/gpu_ab.sh ${TAG}_roll || exit 1
VARIANTS="${RV:-prev main}" PARITY=0 REPS=3 ARGS="--mode step --steps 2000 --warmup 100" bash tools/gpu_ab.sh ${TAG}_step || exit 1
TAG=${TAG}_tail bash tools/gpu_tail.sh || exit 1
