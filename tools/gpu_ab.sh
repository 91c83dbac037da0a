#!/bin/bash
# A/B of library builds (tools/variants.py) in one session: a full-size parity
# check per variant, then interleaved bench repeats.
#   VARIANTS="main rblk64" REPS=3 ARGS="--steps 40 --warmup 5" bash tools/gpu_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-ab}
for v in ${VARIANTS:-main}; do
  if [ "${PARITY:-1}" = 1 ]; then
    BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_full_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "rollout_matches or step_path" > gpurun_out/${TAG}_pytest_$v.log 2>&1
    rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
    [ $rc -eq 0 ] || exit $rc
  fi
done
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-main}; do
    BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so timeout -k 10 120 python bench.py --no-cpu-baseline ${ARGS:---steps 40 --warmup 5} > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$r.json'));print('$v', $r, '%.3e'%d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
