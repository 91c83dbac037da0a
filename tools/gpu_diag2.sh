#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-d2}
timeout -k 10 900 python -m pytest tests/test_gpu_env_parity.py tests/test_gpu_solver_stress.py tests/test_gpu_single_env.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
BB_LANE_BUDGET=0 STEPS=60 timeout -k 10 300 python tools/diag_solver.py > gpurun_out/${TAG}_diag_b0.json 2> gpurun_out/${TAG}_diag.err || exit 1
WARM=40 STEPS=60 N=65536 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_st.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/${TAG}_st.json'));print('default', round(d['us_mean'],1))"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
