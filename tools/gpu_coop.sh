#!/bin/bash
# bb_step workgroup-cooperative search: parity (crowded boards, Lemire rejections, full-size step path),
# the T = 1 tail diagnostics, step-mode A/B of the coop variants, rollout A/B against the previous build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-coop}
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver_stress.py tests/test_gpu_full_parity.py tests/test_gpu_env_parity.py tests/test_gpu_single_env.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "not rollout_matches and not shard_unseeded" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=${TAG}_tail bash tools/gpu_tail.sh || exit 1
VARIANTS="${SVARS:-coop0 main coopr2 coopkw8 coopkw16}" PARITY=0 REPS=${REPS:-2} ARGS="--mode step --steps 2000 --warmup 100" bash tools/gpu_ab.sh ${TAG}_step || exit 1
VARIANTS="prev main" PARITY=0 REPS=2 ARGS="--steps 640 --warmup 64" bash tools/gpu_ab.sh ${TAG}_roll || exit 1
