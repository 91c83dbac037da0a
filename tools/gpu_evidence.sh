#!/bin/bash
# One GPU call of round evidence: smoke(), the whole -m gpu suite (or FILES), the default bench line, then
# (PROFILE=1) rocprofv3 kernel stats + PMC traffic (tools/gpu_profile.sh) and the SQ instruction-issue
# record of the bench kernel (separate --pmc passes -> TAG_sq.json, the roofline.valu source).
# usage: tools/gpu_evidence.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-ev}; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_default_bench.json 2> gpurun_out/${TAG}_default_bench.err || { tail gpurun_out/${TAG}_default_bench.err; exit 1; }
cat gpurun_out/${TAG}_default_bench.json
[ "${PROFILE:-0}" = 1 ] || exit 0
bash tools/gpu_profile.sh "$TAG" || exit 1
NODIAG=1 ARGS="--steps 20 --warmup 10 --no-cpu-baseline" bash tools/gpu_sq_async.sh "${TAG}sq" || exit 1
python3 tools/sq_summary.py gpurun_out "${TAG}sq" rollout_async_kernel --json gpurun_out/${TAG}_sq.json --envs 65536 --steps-per-launch 128 > /dev/null
cat gpurun_out/${TAG}_sq.json
