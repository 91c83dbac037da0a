#!/bin/bash
# parity subset + step timing + bench (+ optional rocprof kernel stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-q}
timeout -k 10 900 python -m pytest ${TESTS:-tests/test_gpu_solver_stress.py tests/test_gpu_env_parity.py tests/test_gpu_single_env.py} -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -m5 -B2 -A20 "Error\|assert" gpurun_out/pytest_$TAG.log | head -60; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench', d['value'], d['roofline']['kernel_avg_ms'])"
for n in ${NS:-4096}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --envs $n > gpurun_out/bench_${TAG}_$n.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$n.json'));print('bench n=$n', d['value'], d['roofline']['kernel_avg_ms'])"
done
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
  grep "bb::" "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG/run_kernel_stats.csv" | cut -c1-40,100-200
fi
for kv in ${EXTRA:-}; do
  timeout -k 10 120 env $kv python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/bench_${TAG}_x.json" 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('$GRAFT_REPO_ROOT/gpurun_out/bench_${TAG}_x.json'));print('bench $kv', d['value'], d['roofline']['kernel_avg_ms'])"
done
