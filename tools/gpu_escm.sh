#!/bin/bash
# Escalate kernel with the multi-env hand search: full -m gpu suite on the
# default build, env parity on the group-size variants, step times per variant,
# then the step-mode bench line.
# Variant libraries (flags in tools/variants.py), built on the CPU beforehand:
#   python tools/variants.py build esc0 escg16 escg32
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-escm}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for v in escg16 escg32; do
  BBVEC_LIB=tools/variants/libbbvec_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_env_parity.py tests/test_gpu_solver_stress.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc"; tail -2 gpurun_out/${TAG}_pytest_$v.log
  [ $rc -eq 0 ] || exit $rc
done
st() { # name, env...
  local name=$1; shift
  env "$@" WARM=40 STEPS=100 timeout -k 10 180 python tools/step_times.py > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -20 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['us_mean'],1), round(d['us_median'],1), round(d['us_max'],1))"
}
st esc0 N=65536 BBVEC_LIB=tools/variants/libbbvec_esc0.so || exit 1
st main N=65536 || exit 1
st g16 N=65536 BBVEC_LIB=tools/variants/libbbvec_escg16.so || exit 1
st g32 N=65536 BBVEC_LIB=tools/variants/libbbvec_escg32.so || exit 1
timeout -k 10 300 python bench.py --mode step --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/${TAG}_bench_step.json 2> gpurun_out/${TAG}_bench_step.err || exit 1
cat gpurun_out/${TAG}_bench_step.json
