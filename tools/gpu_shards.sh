#!/bin/bash
# The bench kernel split over S env handles on S HIP streams (bench.py --shards S): one launch's tail -- the
# slowest workgroup of 256 -- is filled by the other streams' next launches.  REPS interleaved repeats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sh}
for r in $(seq 1 ${REPS:-2}); do
  for s in ${SHARDS:-1 2 4}; do
    timeout -k 10 200 python bench.py --shards $s ${BENCH_ARGS:---steps 200 --warmup 20} --no-cpu-baseline > gpurun_out/${TAG}_s${s}_$r.json 2> gpurun_out/${TAG}_s${s}_$r.err || { tail -5 gpurun_out/${TAG}_s${s}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('shards', sys.argv[2], 'rep', sys.argv[3], d['value'], d['ms_per_step'], d['roofline']['frac'])" gpurun_out/${TAG}_s${s}_$r.json $s $r
  done
done
