set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?
echo "bench rc=$rc"; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err
exit $rc
