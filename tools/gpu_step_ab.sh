#!/bin/bash
# bb_step (step_fused_kernel) A/B of library builds: parity of each variant on the step-path suites, then
# REPS interleaved bench lines in step mode.  VARIANTS="main sq1" REPS=3 bash tools/gpu_step_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sab}; R=$GRAFT_REPO_ROOT
libof() { [ "$1" = main ] && echo "$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so" || echo "$R/build/ab/libbbvec_$1.so"; }
for v in ${VARIANTS:-main}; do
  BBVEC_LIB=$(libof $v) timeout -k 10 600 python -u -m pytest tests/test_gpu_env_parity.py tests/test_gpu_solver_stress.py \
    tests/test_gpu_full_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "step or vec_env or crowded or lemire or hard" > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
  [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit $rc; }
done
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-main}; do
    BBVEC_LIB=$(libof $v) timeout -k 10 120 python bench.py --no-cpu-baseline --mode step --steps 2000 --warmup 100 > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$r.json'));print('$v', $r, '%.4e'%d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
