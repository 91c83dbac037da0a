#!/bin/bash
# rollout_async_kernel (search waves) on the GPU: rollout parity first, then an interleaved A/B of
# library builds (tools/variants.py) on the default bench line.
#   VARIANTS="main sync" REPS=2 bash tools/gpu_async.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-async}
timeout -k 10 400 python -u -m pytest tests/test_gpu_rollout.py tests/test_gpu_full_parity.py -m gpu -x -v \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_pytest.log; exit $rc; }
for v in ${VARIANTS:-main sync}; do  # full-size rollout parity of every variant
  [ "$v" = main ] && continue
  BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_full_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "rollout_matches" > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
  [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-main sync}; do
    lib=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so
    [ "$v" = main ] && lib=$GRAFT_REPO_ROOT/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
    BBVEC_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline ${ARGS:---steps 40 --warmup 5} > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$r.json'));print('$v', $r, '%.3e'%d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
