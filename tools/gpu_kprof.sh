#!/bin/bash
# per-kernel durations (rocprofv3 kernel trace) for several env counts / modes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-kp}
R=$GRAFT_REPO_ROOT
for cfg in ${CFGS:-65536:head 4096:head 65536:cur}; do
  n=${cfg%%:*}; lib=${cfg#*:}
  L=$R/tools/variants/libbbvec_$lib.so; [ "$lib" = cur ] && L=$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
  cd /tmp && BBVEC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_${n}_$lib" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --envs $n --steps 200 --warmup 40 > "$R/gpurun_out/${TAG}_${n}_$lib.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_${n}_$lib.log"; exit 1; }
  f=$(find "$R/gpurun_out/${TAG}_${n}_$lib" -name "*kernel_stats.csv" | head -1)
  echo "== $n $lib"; python -c "import json;d=json.load(open('$R/gpurun_out/${TAG}_${n}_$lib.log'.replace('.log','.log')))" 2>/dev/null; grep -o '"value": [0-9.]*\|"kernel_avg_ms": [0-9.]*' "$R/gpurun_out/${TAG}_${n}_$lib.log" | tr '\n' ' '; echo
  grep "bb::" "$f" | cut -d, -f1-4 | sed 's/(bb::EnvDev[^"]*//'
done
