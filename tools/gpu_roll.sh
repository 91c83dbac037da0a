#!/bin/bash
# rollout parity tests + bench in both modes + T / variant sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-roll}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_rollout.py} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ]; then grep -m5 -B5 -A30 "Error\|assert" gpurun_out/pytest_$TAG.log | head -80; exit $rc; fi
for cfg in ${CFGS:-step:1 rollout:10 rollout:50 rollout:200}; do
  set -- ${cfg/:/ }
  timeout -k 10 200 python bench.py --no-cpu-baseline --mode $1 --rollout-len $2 --steps 400 --warmup 40 > gpurun_out/bench_${TAG}_$1_$2.json 2> gpurun_out/bench_${TAG}.err || { tail -5 gpurun_out/bench_${TAG}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_$1_$2.json'));print('$1 T=$2', d['value'], d['roofline']['kernel_avg_ms'])"
done
for lib in ${LIBS:-}; do
  for T in ${LTS:-128}; do
    BBVEC_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --mode rollout --rollout-len $T --steps 400 --warmup 40 > gpurun_out/bench_${TAG}_x.json 2>>gpurun_out/bench_${TAG}.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_x.json'));print('$lib T=$T', d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
for kv in ${EXTRA:-}; do
  env $kv timeout -k 10 200 python bench.py --no-cpu-baseline --mode rollout --rollout-len 200 --steps 400 --warmup 40 > gpurun_out/bench_${TAG}_x.json 2>>gpurun_out/bench_${TAG}.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_x.json'));print('$kv T=200', d['value'], d['roofline']['kernel_avg_ms'])"
done
for sh in ${SHARDS:-}; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --shards $sh --steps 1280 --warmup 128 > gpurun_out/bench_${TAG}_x.json 2>>gpurun_out/bench_${TAG}.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_x.json'));print('shards=$sh', d['value'], d['roofline']['kernel_avg_ms'])"
done
for cfg in ${SHT:-}; do
  set -- ${cfg/:/ }
  timeout -k 10 200 python bench.py --no-cpu-baseline --shards $1 --rollout-len $2 --steps 1280 --warmup 128 > gpurun_out/bench_${TAG}_x.json 2>>gpurun_out/bench_${TAG}.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_x.json'));print('shards=$1 T=$2', d['value'], d['roofline']['kernel_avg_ms'])"
done
