#!/bin/bash
# A/B of the bf16 optimizer step (tools/prof_update.py) across library builds copied to build/ab/ (tools/variants/
# does not travel to the GPU box), interleaved, after the optimizer / PPO-kernel GPU tests of each build.
#   VARIANTS="main hrx" REPS=3 bash tools/gpu_update_ab2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-upd}; R=$GRAFT_REPO_ROOT
libof() { [ "$1" = main ] && echo "$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so" || echo "$R/build/ab/libbbvec_$1.so"; }
for v in ${VARIANTS:-main}; do
  BBVEC_LIB=$(libof $v) timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_kernels.py tests/test_gpu_optim.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in $(seq 1 ${REPS:-3}); do
  for v in ${VARIANTS:-main}; do
    BBVEC_LIB=$(libof $v) timeout -k 10 120 python tools/prof_update.py --batch 2048 --steps 200 ${PU_ARGS:-} > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    echo "$v $r $(cat gpurun_out/${TAG}_${v}_$r.json)"
  done
done
[ "${KT:-0}" = 1 ] || exit 0
cd /tmp || exit 1
for v in ${VARIANTS:-main}; do
  BBVEC_LIB=$(libof $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_kt_$v" -o run --output-format csv -- python3 "$R/tools/prof_update.py" --batch 2048 --steps 50 > "$R/gpurun_out/${TAG}_kt_$v.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_kt_$v.log"; exit 1; }
  python3 "$R/tools/prof_update.py" --summarize "$(find "$R/gpurun_out/${TAG}_kt_$v" -name '*kernel_trace.csv' | sort | tail -1)" --steps 50 > "$R/gpurun_out/${TAG}_kernels_$v.txt" 2>&1
  head -24 "$R/gpurun_out/${TAG}_kernels_$v.txt" | cut -c1-140
done
