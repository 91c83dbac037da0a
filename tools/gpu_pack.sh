#!/bin/bash
# Escalation pass-schedule sweep (tuning): parity first, then per-step time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pack}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest ${TESTS:-tests/test_gpu_solver_stress.py tests/test_gpu_eval.py} -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
for pk in ${PACKS:-1,0 1,32 2,32 4,32 8,32 32,32 1,8 2,16}; do
  f=${pk%,*}; x=${pk#*,}
  BB_PACK_FIRST=$f BB_PACK_NEXT=$x N=65536 WARM=40 STEPS=60 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_$f-$x.json 2> gpurun_out/${TAG}_$f-$x.err || { tail -20 gpurun_out/${TAG}_$f-$x.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$f-$x.json'));print('pack $pk us', round(d['us_mean'],1), round(d['us_median'],1), round(d['us_max'],1))"
done
