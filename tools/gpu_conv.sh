#!/bin/bash
# HIP board convolutions: parity tests, then the microbench vs MIOpen.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-conv}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ${KSEL:+-k "$KSEL"} ${PYARGS:-} > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | tail -30
[ $rc -eq 0 ] || [ "${BENCH_ANYWAY:-0}" = 1 ] || exit $rc
timeout -k 10 200 python tools/bench_conv.py ${BARGS:-} > gpurun_out/${TAG}_bench.jsonl 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.jsonl
