#!/bin/bash
# Config 3 (full PPO, bf16 autocast) with the HIP board convolutions vs MIOpen's
# (BB_HIP_CONV=0), after the conv parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-c3conv}
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "conv pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for hc in ${HC:-1 0}; do
  BB_HIP_CONV=$hc timeout -k 10 400 python tools/bench_ppo.py --envs ${ENVS:-65536} --update-steps 200 --autocast bf16 ${BARGS:-} > gpurun_out/${TAG}_hc$hc.json 2> gpurun_out/${TAG}_hc$hc.err || { tail -5 gpurun_out/${TAG}_hc$hc.err; exit 1; }
  echo "hip_conv=$hc $(cat gpurun_out/${TAG}_hc$hc.json)"
done
