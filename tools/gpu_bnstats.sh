#!/bin/bash
# BatchNorm statistics from the convolution epilogue (BB_CONV_BN_STATS): parity tests, then the bf16
# optimizer step with and without it (tools/bench_ppo.py, interleaved repeats).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-bns}
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_optim.py tests/test_gpu_ppo_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_pytest.log; exit $rc; }
for r in $(seq 1 ${REPS:-2}); do
  for v in 1 0; do
    BB_CONV_BN_STATS=$v timeout -k 10 200 python tools/bench_ppo.py --envs 8192 --update-steps 300 --autocast bf16 > gpurun_out/${TAG}_s${v}_$r.json 2>gpurun_out/${TAG}_s${v}_$r.err || { tail -5 gpurun_out/${TAG}_s${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_s${v}_$r.json'));print('stats=$v', $r, d['update_step_ms'])"
  done
done
