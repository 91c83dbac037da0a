#!/bin/bash
# A/B of library builds (tools/variants.py) on the config-3 optimizer step (bf16 autocast):
#   VARIANTS="main bnr1024" REPS=2 bash tools/gpu_upd_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-updab}
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-main}; do
    lib=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so
    [ "$v" = main ] && lib=$GRAFT_REPO_ROOT/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
    BBVEC_LIB=$lib timeout -k 10 200 python tools/bench_ppo.py --envs 8192 --update-steps 300 --autocast bf16 > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$r.json'));print('$v', $r, d['update_step_ms'])"
  done
done
