#!/bin/bash
# Round-3 check: the GPU parity suites touched by this round's changes, then
# the step-mode bench (bb_step at 65,536 envs) and its HBM traffic (two PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03a}
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_ppo_update_oracle.py tests/test_gpu_train.py tests/test_gpu_env_parity.py tests/test_gpu_full_parity.py tests/test_gpu_rollout.py tests/test_gpu_single_env.py tests/test_gpu_train_rollout_oracle.py} -m gpu -v -s --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || { [ "${CONT:-0}" = 1 ] && [ $rc -eq 1 ]; } || exit $rc
R="$GRAFT_REPO_ROOT"
for k in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --mode step --steps 2000 --warmup 100 > gpurun_out/${TAG}_step_$k.json 2>gpurun_out/${TAG}_step_$k.err || { tail -5 gpurun_out/${TAG}_step_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_step_$k.json'));print('step', '%.3e'%d['value'], d['roofline']['kernel_avg_ms'])"
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/${TAG}_roll_$k.json 2>gpurun_out/${TAG}_roll_$k.err || { tail -5 gpurun_out/${TAG}_roll_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_roll_$k.json'));print('rollout', '%.3e'%d['value'], d['roofline']['kernel_avg_ms'])"
done
cd /tmp || exit 1
A="--no-cpu-baseline --mode step --steps 400 --warmup 50"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_fetch" -o run --output-format csv -- python "$R/bench.py" $A > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_write" -o run --output-format csv -- python "$R/bench.py" $A > "$R/gpurun_out/${TAG}_write.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_write.log"; exit 1; }
python "$R/tools/pmc_traffic.py" "$R/gpurun_out/${TAG}_fetch" "$R/gpurun_out/${TAG}_write" --envs 65536 --kernels rollout_kernel --steps-per-launch 1 --out "$R/gpurun_out/${TAG}_pmc_step.json"
cat "$R/gpurun_out/${TAG}_pmc_step.json"
