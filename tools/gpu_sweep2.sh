#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sw}
st() { # name, env...
  local name=$1; shift
  env "$@" WARM=40 STEPS=60 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -20 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['us_mean'],1), round(d['us_median'],1), round(d['us_max'],1))"
}
st def N=65536 || exit 1
st b16 N=65536 BB_LANE_BUDGET=16 || exit 1
st b12 N=65536 BB_LANE_BUDGET=12 || exit 1
st n4k N=4096 || exit 1
st n1k N=1024 || exit 1
st n16k N=16384 || exit 1
st ns65k N=65536 BB_DEBUG_MODE=1 || exit 1
st ns16k N=16384 BB_DEBUG_MODE=1 || exit 1
st ns4k N=4096 BB_DEBUG_MODE=1 || exit 1
st ns262k N=262144 BB_DEBUG_MODE=1 || exit 1
