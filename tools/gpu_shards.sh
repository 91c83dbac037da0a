#!/bin/bash
# shard / stream sweep of the rollout and step benches (tail overlap across HIP streams)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sh; export TMPDIR=/tmp
TAG=${1:-sh}
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/sh/${TAG}_$nm.json 2>>gpurun_out/sh/${TAG}.err || { tail -5 gpurun_out/sh/${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sh/${TAG}_$nm.json'));print('$nm', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], flush=True)"
}
for cfg in ${CFGS:-r:1:128 r:2:128 r:4:128 r:8:128 r:1:256 r:1:512 s:1:1 s:2:1 s:4:1 s:8:1 s:16:1}; do
  IFS=: read m sh T <<< "$cfg"
  if [ $m = r ]; then run r${sh}_$T --shards $sh --rollout-len $T --steps $((128000 / T)) --warmup 20 || exit 1
  else run s${sh} --mode step --shards $sh --steps 4000 --warmup 200 || exit 1; fi
done
