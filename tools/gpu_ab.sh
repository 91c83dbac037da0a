#!/bin/bash
# A/B benchmark of two library builds in one session (alternating, 3 rounds each).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
for r in 1 2 3; do
  for v in ${VARIANTS:-A B}; do
    BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 400 > gpurun_out/${TAG}_$v.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_$v.json'));print('$v', round(d['value']/1e6,1), d['roofline']['kernel_avg_ms'])"
  done
done
