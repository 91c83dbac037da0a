#!/bin/bash
# Round-6 end evidence in one GPU call (the shipped build): smoke(), the whole -m gpu suite, the default bench line
# and the driver's own command, rocprofv3 kernel stats + two PMC passes of the bench kernel (-> pmc json), the SQ
# counter passes (-> sq json), the bb_step PMC, and the bf16 optimizer step's timing + kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06end}; R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_driver_bench.json 2> gpurun_out/${TAG}_driver_bench.err || { tail gpurun_out/${TAG}_driver_bench.err; exit 1; }
echo "driver command: $(python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_driver_bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])")"
ARGS="--steps 200 --warmup 20" bash tools/gpu_profile.sh "$TAG" > gpurun_out/${TAG}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile.log; exit 1; }
tail -3 gpurun_out/${TAG}_profile.log
NODIAG=1 ARGS="--steps 20 --warmup 10 --no-cpu-baseline" bash tools/gpu_sq_async.sh "${TAG}sq" > gpurun_out/${TAG}_sqrun.log 2>&1 || { tail -20 gpurun_out/${TAG}_sqrun.log; exit 1; }
python3 tools/sq_summary.py gpurun_out "${TAG}sq" rollout_async_kernel --json gpurun_out/${TAG}_sq.json --envs 65536 --steps-per-launch 128 > /dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_sq.json'));print('valu', d.get('valu_insts_per_launch'), d.get('build_id'))"
ARGS="--mode step --steps 2000 --warmup 100 --no-cpu-baseline" PMC_ARGS="--kernels step_fused_kernel --steps-per-launch 1" bash tools/gpu_profile.sh "${TAG}_step" > gpurun_out/${TAG}_step_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_step_profile.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_step_bench.json'));print('bb_step', d['value'])"
for r in 1 2; do
  timeout -k 10 180 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/${TAG}_pu_$r.json 2> gpurun_out/${TAG}_pu_$r.err || { tail -5 gpurun_out/${TAG}_pu_$r.err; exit 1; }
  tail -1 gpurun_out/${TAG}_pu_$r.json
done
cd /tmp || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_pukt" -o run --output-format csv -- python3 "$R/tools/prof_update.py" --batch 2048 --steps 50 > "$R/gpurun_out/${TAG}_pukt.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_pukt.log"; exit 1; }
python3 "$R/tools/prof_update.py" --summarize "$(find "$R/gpurun_out/${TAG}_pukt" -name '*kernel_trace.csv' | sort | tail -1)" --steps 50 > "$R/gpurun_out/${TAG}_update_kernels.txt" 2>&1
head -1 "$R/gpurun_out/${TAG}_update_kernels.txt"
