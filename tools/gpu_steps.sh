#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-st}
for n in 65536 16384 262144; do
  N=$n WARM=${WARM:-40} STEPS=${STEPS:-60} timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_$n.json 2> gpurun_out/${TAG}_$n.err || { tail -20 gpurun_out/${TAG}_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$n.json'));print($n, d['us_mean'], d['us_median'], d['us_max']); print(d['per_step'][:30])"
done
