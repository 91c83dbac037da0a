#!/bin/bash
# The first FC layer's forward on bb_linear_relu_forward vs hipBLASLt + bb_dropout_forward (BB_FC_GEMM=0):
# the Linear / optimizer / PPO-kernel GPU suites, then REPS interleaved bf16 optimizer-step timings of both, then
# one kernel trace of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fc}; R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_tail.py tests/test_gpu_optim.py tests/test_gpu_ppo_kernels.py tests/test_gpu_network_oracle.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; }
for r in $(seq 1 ${REPS:-3}); do
  for v in 1 0; do
    BB_FC_GEMM=$v timeout -k 10 120 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/${TAG}_fc${v}_$r.json 2>gpurun_out/${TAG}_fc${v}_$r.err || { tail -5 gpurun_out/${TAG}_fc${v}_$r.err; exit 1; }
    echo "fc$v $r $(cat gpurun_out/${TAG}_fc${v}_$r.json)"
  done
done
cd /tmp || exit 1
for v in 1 0; do
  BB_FC_GEMM=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_kt_$v" -o run --output-format csv -- python3 "$R/tools/prof_update.py" --batch 2048 --steps 50 > "$R/gpurun_out/${TAG}_kt_$v.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_kt_$v.log"; exit 1; }
  python3 "$R/tools/prof_update.py" --summarize "$(find "$R/gpurun_out/${TAG}_kt_$v" -name '*kernel_trace.csv' | sort | tail -1)" --steps 50 > "$R/gpurun_out/${TAG}_kernels_$v.txt" 2>&1
  head -1 "$R/gpurun_out/${TAG}_kernels_$v.txt"; grep -E "linear_tn|splitk_relu|Cijk|dropout" "$R/gpurun_out/${TAG}_kernels_$v.txt" | cut -c1-150
done
