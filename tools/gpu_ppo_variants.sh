#!/bin/bash
# config-3 update-step timing under MIOpen / layout variants (bf16 autocast)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
run() {  # name, env, args
  env $2 timeout -k 10 400 python tools/bench_ppo.py --envs 8192 --update-steps ${US:-200} $3 > gpurun_out/ppov_$1.json 2> gpurun_out/ppov_$1.err || { tail -5 gpurun_out/ppov_$1.err; return 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ppov_$1.json'));print('$1', d['update_step_ms'], d['update_cnn_tflops'], d['rollout_env_steps_per_s'])"
}
run bf16 "X=1" "--autocast bf16" &&
run bf16_nogemm "MIOPEN_DEBUG_CONV_GEMM=0" "--autocast bf16" &&
run bf16_cl "X=1" "--autocast bf16 --channels-last" &&
run bf16_cl_nogemm "MIOPEN_DEBUG_CONV_GEMM=0" "--autocast bf16 --channels-last" &&
run bf16_find "X=1" "--autocast bf16 --miopen-find" &&
run fp32 "X=1" "" &&
run fp32_nogemm "MIOPEN_DEBUG_CONV_GEMM=0" ""
