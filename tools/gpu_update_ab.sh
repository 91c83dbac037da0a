#!/bin/bash
# A/B of the bf16 optimizer step (tools/prof_update.py, 2,048 samples) across library builds
# (tools/variants.py), interleaved, after the CNN-kernel GPU tests of each build.
#   VARIANTS="main bnu4" REPS=3 bash tools/gpu_update_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-upd}; R=$GRAFT_REPO_ROOT
libof() { [ "$1" = main ] && echo "$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so" || echo "$R/tools/variants/libbbvec_$1.so"; }
for v in ${VARIANTS:-main}; do
  BBVEC_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_kernels.py tests/test_gpu_optim.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-main}; do
    BBVEC_LIB=$(libof $v) timeout -k 10 120 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    echo "$v $r $(cat gpurun_out/${TAG}_${v}_$r.json)"
  done
done
