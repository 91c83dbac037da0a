#!/bin/bash
# Development loop on the GPU box: the whole -m gpu suite, then the default
# rollout bench line and the step-mode line (no CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-dev}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 180 python bench.py --no-cpu-baseline --steps 400 --warmup 40 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('rollout', '%.4e'%d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
timeout -k 10 180 python bench.py --no-cpu-baseline --mode step --steps 400 --warmup 40 > gpurun_out/${TAG}_bench_step.json 2> gpurun_out/${TAG}_bench_step.err || { tail gpurun_out/${TAG}_bench_step.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_step.json'));print('step', '%.4e'%d['value'], d['roofline']['kernel_avg_ms'])"
