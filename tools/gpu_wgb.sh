set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/wgb; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_env_parity.py tests/test_gpu_rollout.py tests/test_gpu_solver_stress.py tests/test_gpu_full_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/wgb/pytest_env.log 2>&1 || { tail -30 gpurun_out/wgb/pytest_env.log; exit 1; }
tail -2 gpurun_out/wgb/pytest_env.log
VARIANTS="wgb0 main" PARITY=0 REPS=3 ARGS="--mode step --steps 4000 --warmup 200" bash tools/gpu_ab.sh wgb/step || exit 1
VARIANTS="wgb2" PARITY=1 REPS=0 bash tools/gpu_ab.sh wgb/roll || exit 1
VARIANTS="main wgb2" PARITY=0 REPS=3 ARGS="--steps 1000 --warmup 20" bash tools/gpu_ab.sh wgb/roll || exit 1
