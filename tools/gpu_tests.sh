#!/bin/bash
# Selected -m gpu test files (args), then optionally the default bench line: one GPU call.
# usage: tools/gpu_tests.sh TAG "tests/a.py tests/b.py" [bench]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; FILES=$2
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
if [ "$3" = "bench" ]; then
  timeout -k 10 300 python bench.py --steps 1280 --warmup 128 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_bench.json
fi
