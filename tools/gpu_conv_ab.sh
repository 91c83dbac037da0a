#!/bin/bash
# A/B of library builds (tools/variants.py) on the board-convolution microbench:
#   VARIANTS="main cdiag1" bash tools/gpu_conv_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-convab}
for r in $(seq 1 ${REPS:-1}); do
  for v in ${VARIANTS:-main}; do
    lib=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so
    [ "$v" = main ] && lib=$GRAFT_REPO_ROOT/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
    BBVEC_LIB=$lib timeout -k 10 120 python tools/bench_conv.py --shapes ${SHAPES:-128x128} > gpurun_out/${TAG}_${v}_$r.jsonl 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "
import json
for l in open('gpurun_out/${TAG}_${v}_$r.jsonl'):
    d=json.loads(l); print('$v', d['shape'], 'fwd', d['hip_fwd_us'], 'dgrad', d['hip_dgrad_us'], 'wgrad', d['hip_wgrad_us'])"
  done
done
