#!/bin/bash
# bb_step A/B: per library variant the step-mode bench (interleaved repeats) and its HBM
# bytes per env-step from two PMC passes:  VARIANTS="main seager" bash tools/gpu_step_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-stepab}; R=$GRAFT_REPO_ROOT
VARIANTS="${VARIANTS:-main}" PARITY=${PARITY:-0} REPS=${REPS:-3} ARGS="--mode step --steps 2000 --warmup 100" bash tools/gpu_ab.sh $TAG || exit 1
cd /tmp || exit 1
A="--no-cpu-baseline --mode step --steps 400 --warmup 50"
for v in ${VARIANTS:-main}; do
  L=$R/tools/variants/libbbvec_$v.so
  BBVEC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_fetch" -o run --output-format csv -- python "$R/bench.py" $A > "$R/gpurun_out/${TAG}_${v}_fetch.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_${v}_fetch.log"; exit 1; }
  BBVEC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_${v}_write" -o run --output-format csv -- python "$R/bench.py" $A > "$R/gpurun_out/${TAG}_${v}_write.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_${v}_write.log"; exit 1; }
  python "$R/tools/pmc_traffic.py" "$R/gpurun_out/${TAG}_${v}_fetch" "$R/gpurun_out/${TAG}_${v}_write" --envs 65536 --kernels rollout_kernel --steps-per-launch 1 --out "$R/gpurun_out/${TAG}_${v}_pmc.json" > /dev/null || exit 1
  python -c "import json;d=json.load(open('$R/gpurun_out/${TAG}_${v}_pmc.json'));print('$v bytes/env-step', d['bytes_per_env_step'])"
done
