#!/bin/bash
# One GPU session: parity tests, bench line, kernel-trace profile of the bench.
# Usage (via gpurun): bash tools/gpu_run.sh TAG [pytest-args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
shift
TESTS=${*:-tests}
timeout -k 10 900 python -m pytest $TESTS -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -25 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
f=$(find "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12
exit $rc
