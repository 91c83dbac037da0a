#!/bin/bash
# Round 2 probe: why the driver's `bench.py --steps 20 --warmup 5` read 4.4e9
# while the default 200-step run reads ~6.7e9 (one short launch vs many).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
b() { tag=$1; shift; timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > gpurun_out/probe_$tag.json 2> gpurun_out/probe_$tag.err || { tail -5 gpurun_out/probe_$tag.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/probe_$tag.json'));print('$tag', '$*', '%.3e'%d['value'], d['roofline']['kernel_avg_ms'], d['ms_per_step'])"; }
b k20w5 --steps 20 --warmup 5
b k20w5b --steps 20 --warmup 5
b k200w20 --steps 200 --warmup 20
b k1280w128 --steps 1280 --warmup 128
b k128w128 --steps 128 --warmup 128
b k256w256 --steps 256 --warmup 256
b t20 --steps 200 --warmup 20 --rollout-len 20
b t512 --steps 1024 --warmup 512 --rollout-len 512
