#!/bin/bash
# Env-wave vs search-wave share of rollout_async_kernel's SQ counts by difference: the shipped build against a
# diagnostic build that runs every search call twice (tools/variants.py adup; results of the second dropped),
# plus both builds' per-wave call counts (tools/diag_async.py) to normalise per call.
#   bash tools/gpu_sq_split.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sqs}; R=$GRAFT_REPO_ROOT
SET=${SET:-SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY}
cd /tmp || exit 1
for v in main adup; do
  L=$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so; [ $v = main ] || L=$R/tools/variants/libbbvec_$v.so
  BBVEC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc ${SET//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_p1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 10 > "$R/gpurun_out/${TAG}_${v}.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${v}.log"; exit 1; }
  echo "== $v"; python3 "$R/tools/sq_summary.py" "$R/gpurun_out" "${TAG}_${v}" rollout_async_kernel
done
cd "$R" || exit 1
for v in adiag adupdiag; do
  BBVEC_LIB=tools/variants/libbbvec_$v.so timeout -k 10 120 python3 tools/diag_async.py > gpurun_out/${TAG}_diag_$v.json 2> gpurun_out/${TAG}_diag_$v.err || { tail -5 gpurun_out/${TAG}_diag_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_diag_$v.json'))[-1];print('$v', {k: d[k] for k in ('env_iters_per_step','search_calls_per_wave','envs_per_call','cyc_per_call','search_busy_frac')})"
done
