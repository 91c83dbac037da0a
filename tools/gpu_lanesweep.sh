#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ls}
timeout -k 10 900 python -m pytest tests/test_gpu_env_parity.py tests/test_gpu_solver_stress.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -m3 -A30 "Error\|assert" gpurun_out/pytest_$TAG.log | head -60; exit $rc; fi
b() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['value']/1e6,1), d['roofline']['kernel_avg_ms'])"
}
b b16 || exit 1
for q in 1 2 3 4 6; do b q$q BB_LANE_QUICK=$q || exit 1; done
b b8 BB_LANE_BUDGET=8 || exit 1
b b24 BB_LANE_BUDGET=24 || exit 1
