# tests + ablation + diagnostics in one GPU call (diagnostics; not product)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 BUDGETS="${BUDGETS:-0 32 128}" bash tools/gpu_ablate.sh || exit $?
BB_LANE_BUDGET=0 timeout -k 10 300 python tools/diag_solver.py > gpurun_out/diag_b0.json 2> gpurun_out/diag_b0.err || exit $?
python -c "import json;d=json.load(open('gpurun_out/diag_b0.json'));d.pop('worst');print(json.dumps(d))"
