#!/bin/bash
# Convolution kernels: GPU tests, forward / data-gradient timings (tools/bench_conv.py) of the shipped build
# against VARIANTS, the bf16 optimizer step of each (tools/prof_update.py) and a rocprofv3 kernel trace of
# the shipped build's step (per-kernel breakdown: tools/prof_update.py --summarize).
#   VARIANTS="cws0" bash tools/gpu_conv_ws.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-cws}; R=$GRAFT_REPO_ROOT
for v in main ${VARIANTS:-}; do
  L=$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so; [ $v = main ] || L=$R/tools/variants/libbbvec_$v.so
  BBVEC_LIB=$L timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_optim.py ${TESTS:-} -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc $(tail -1 gpurun_out/${TAG}_pytest_$v.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/${TAG}_pytest_$v.log; exit $rc; }
done
for r in 1 2; do
  for v in main ${VARIANTS:-}; do
    L=$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so; [ $v = main ] || L=$R/tools/variants/libbbvec_$v.so
    BBVEC_LIB=$L timeout -k 10 120 python tools/bench_conv.py --shapes 128x128,64x128 > gpurun_out/${TAG}_conv_${v}_$r.json 2>/dev/null || { tail -5 gpurun_out/${TAG}_conv_${v}_$r.json; exit 1; }
    echo "$v $r conv: $(python -c "import json;[print(json.dumps({k: d[k] for k in d if 'hip' in k or k=='shape'}), end=' ') for d in map(json.loads, open('gpurun_out/${TAG}_conv_${v}_$r.json'))]")"
    BBVEC_LIB=$L timeout -k 10 120 python tools/prof_update.py --batch 2048 --steps 100 > gpurun_out/${TAG}_pu_${v}_$r.json 2>gpurun_out/${TAG}_pu_${v}_$r.err || { tail -5 gpurun_out/${TAG}_pu_${v}_$r.err; exit 1; }
    echo "$v $r update: $(cat gpurun_out/${TAG}_pu_${v}_$r.json)"
  done
done
cd /tmp || exit 1
BBVEC_LIB=${PROF_LIB:-$R/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so} timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_pukt" -o run --output-format csv -- python3 "$R/tools/prof_update.py" --batch 2048 --steps 50 > "$R/gpurun_out/${TAG}_pukt.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_pukt.log"; exit 1; }
python3 "$R/tools/prof_update.py" --summarize "$(find "$R/gpurun_out/${TAG}_pukt" -name '*kernel_trace.csv' | sort | tail -1)" --steps 50 > "$R/gpurun_out/${TAG}_pu_kernels.txt" 2>&1; head -24 "$R/gpurun_out/${TAG}_pu_kernels.txt"
exit 0
