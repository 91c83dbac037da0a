#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-e2}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then exit $rc; fi
st() { # name, env...
  local name=$1; shift
  env "$@" WARM=40 STEPS=60 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -20 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['us_mean'],1), round(d['us_median'],1), round(d['us_max'],1))"
}
st def N=65536 || exit 1
st hf20 N=65536 BB_HARD_FILL=20 || exit 1
st hf34 N=65536 BB_HARD_FILL=34 || exit 1
st hf64 N=65536 BB_HARD_FILL=65 || exit 1
st w6 N=65536 BB_ESC_WAVES_PER_CU=6 || exit 1
st w24 N=65536 BB_ESC_WAVES_PER_CU=24 || exit 1
st b16 N=65536 BB_LANE_BUDGET=16 || exit 1
st n16k N=16384 || exit 1
st n4k N=4096 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
cat gpurun_out/bench_$TAG.json
