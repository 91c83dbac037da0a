#!/bin/bash
# Escalate-kernel variants on top of the multi-env search: jump table in LDS,
# 128-thread blocks.  Env parity + solver stress per variant, then step times.
# Variant libraries (flags in tools/variants.py), built on the CPU beforehand:
#   python tools/variants.py build escj escjb128 escb128
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-escj}
for v in escj escjb128 escb128; do
  BBVEC_LIB=tools/variants/libbbvec_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_env_parity.py tests/test_gpu_solver_stress.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -1 gpurun_out/${TAG}_pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
st() { # name, env...
  local name=$1; shift
  env "$@" WARM=40 STEPS=200 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -20 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['us_mean'],1), round(d['us_median'],1), round(d['us_max'],1))"
}
for rep in 1 2; do
st main$rep N=65536 || exit 1
st j$rep N=65536 BBVEC_LIB=tools/variants/libbbvec_escj.so || exit 1
st jb128_$rep N=65536 BBVEC_LIB=tools/variants/libbbvec_escjb128.so || exit 1
st b128_$rep N=65536 BBVEC_LIB=tools/variants/libbbvec_escb128.so || exit 1
done
