#!/bin/bash
# BatchNorm kernel tests + micro-benchmark + update-step timing in both layouts
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "batchnorm" > gpurun_out/pytest_bn.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_bn.log; [ $rc -eq 0 ] || { grep -m2 -B5 -A30 "Error\|assert" gpurun_out/pytest_bn.log | head -60; exit $rc; }
timeout -k 10 200 python tools/bench_bn.py 2>/dev/null || exit 1
for a in "--autocast bf16" "--autocast bf16 --channels-last" "--autocast none" "--autocast none --channels-last"; do
  timeout -k 10 200 python tools/prof_update.py $a 2>/dev/null || exit 1
done
