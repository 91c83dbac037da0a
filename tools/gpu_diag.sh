set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_env_parity.py tests/test_gpu_solver_stress.py -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/diag_solver.py > gpurun_out/diag.json 2> gpurun_out/diag.err || exit $?
timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/b.json 2>/dev/null || exit $?
python -c "import json;d=json.load(open('gpurun_out/b.json'));print('bench', d['value'], d['roofline']['kernel_avg_ms'])"
