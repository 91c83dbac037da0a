#!/bin/bash
# A/B of rollout library builds (tools/variants.py) on the bench kernel, in one GPU call:
#   1. parity of every variant (async rare paths subset, long-horizon rollout, full-size C-oracle rollout);
#   2. REPS interleaved repeats of the bench line (1,280 steps);
#   3. per variant one rocprofv3 WRITE_SIZE and one FETCH_SIZE pass (HBM traffic per env-step).
#   VARIANTS="main aw8" REPS=3 bash tools/gpu_ab_async.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-ab}; R=$GRAFT_REPO_ROOT
# a variant is a library name (tools/variants.py; "main" = the shipped build), optionally followed by
# runtime settings: "main:BB_PACK_FIRST=4:BB_PACK_NEXT=16"
libof() { local n=${1%%:*}; [ "$n" = main ] && echo "$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so" || echo "$R/build/ab/libbbvec_$n.so"; }
envof() { local e=${1#*:}; [ "$e" = "$1" ] && echo "" || echo "${e//:/ }"; }
for v in ${VARIANTS:-main}; do
  env $(envof $v) BBVEC_LIB=$(libof $v) timeout -k 10 600 python -u -m pytest tests/test_gpu_full_parity.py tests/test_gpu_rollout.py \
    tests/test_gpu_async_rare_paths.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    -k "${PK:-rollout_matches or long_horizon or many_workgroups or lemire}" > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"
  [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit $rc; }
done
for d in ${DIAG:-}; do  # diagnostic builds (BB_ASYNC_DIAG=1): per-wave counters (tools/diag_async.py)
  BBVEC_LIB=$R/build/ab/libbbvec_$d.so timeout -k 10 120 python3 tools/diag_async.py > gpurun_out/${TAG}_diag_$d.json 2> gpurun_out/${TAG}_diag_$d.err || { tail -5 gpurun_out/${TAG}_diag_$d.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_diag_$d.json'))[-1];print('$d', {k: d[k] for k in ('env_iters_per_step','env_iters_max','env_wave_cyc_mean','env_wave_cyc_max','env_wave_cyc_by_index','slowest_index_share','wg_cyc_mean_of_max','cyc_per_call','envs_per_call')})"
done
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-main}; do
    env $(envof $v) BBVEC_LIB=$(libof $v) timeout -k 10 120 python bench.py --no-cpu-baseline ${ARGS:---steps 1280 --warmup 128} > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$r.json'));print('$v', $r, '%.4e'%d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
cd /tmp || exit 1
if [ -n "$SQPASS" ]; then  # one SQ counter pass per variant (e.g. SQPASS=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE)
  for v in ${VARIANTS:-main}; do
    env $(envof $v) BBVEC_LIB=$(libof $v) timeout -s KILL 120 rocprofv3 --pmc ${SQPASS//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_sq_p1" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 10 > "$R/gpurun_out/${TAG}_${v}_sq.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${v}_sq.log"; exit 1; }
    echo "== $v"; python3 "$R/tools/sq_summary.py" "$R/gpurun_out" "${TAG}_${v}_sq" rollout_async_kernel
  done
fi
[ -n "$NOPMC" ] && exit 0
for v in ${VARIANTS:-main}; do
  for c in WRITE_SIZE FETCH_SIZE; do
    env $(envof $v) BBVEC_LIB=$(libof $v) timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_$c" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 10 > "$R/gpurun_out/${TAG}_${v}_$c.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${v}_$c.log"; exit 1; }
  done
  python3 "$R/tools/pmc_traffic.py" "$R/gpurun_out/${TAG}_${v}_FETCH_SIZE" "$R/gpurun_out/${TAG}_${v}_WRITE_SIZE" --envs 65536 --kernels rollout_async_kernel --steps-per-launch 128 --out "$R/gpurun_out/${TAG}_${v}_pmc.json" > /dev/null || exit 1
  python3 -c "import json;d=json.load(open('$R/gpurun_out/${TAG}_${v}_pmc.json'));print('$v pmc', {k: d[k] for k in d if 'per_env_step' in k})"
done
