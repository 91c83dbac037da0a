#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-lane}
for b in ${BUDGETS:-0 12 16 24 40 64}; do
  BB_LANE_BUDGET=$b timeout -k 10 180 python tools/diag_lane.py > gpurun_out/${TAG}_diag_b$b.json 2> gpurun_out/${TAG}_diag_b$b.err || { tail -20 gpurun_out/${TAG}_diag_b$b.err; exit 1; }
  cat gpurun_out/${TAG}_diag_b$b.json
  BB_LANE_BUDGET=$b N=65536 WARM=40 STEPS=60 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_st_b$b.json 2> gpurun_out/${TAG}_st_b$b.err || { tail -20 gpurun_out/${TAG}_st_b$b.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_st_b$b.json'));print('budget $b us', d['us_mean'], d['us_median'], d['us_max'])"
done
