#!/bin/bash
# BatchNorm partials layout: parity (BatchNorm / network / optimizer tests), update-step A/B, and the pending
# bb_step multi-pass A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-bnp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_kernels.py tests/test_gpu_optim.py tests/test_gpu_conv.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="prev main bnr1024 bnr2048" REPS=2 bash tools/gpu_upd_ab.sh ${TAG}_upd || exit 1
VARIANTS="main mp2 mp4 mp6" PARITY=0 REPS=2 ARGS="--mode step --steps 2000 --warmup 100" bash tools/gpu_ab.sh ${TAG}_mps || exit 1
