# Budget / size ablation of the step kernels (diagnostics; not part of the product).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
run() { # name, env assignments...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --warmup 20 ${BENCH_ARGS:-} > gpurun_out/abl_$name.json 2> gpurun_out/abl_$name.err || return $?
  python -c "import json;d=json.load(open('gpurun_out/abl_$name.json'));print('$name', d['value'], d['roofline']['kernel_avg_ms'])"
}
for b in ${BUDGETS:-16 64 128 256 512 1024 1000000000}; do
  run b$b BB_LANE_BUDGET=$b || exit $?
done
run nosolve BB_DEBUG_MODE=1 || exit $?
