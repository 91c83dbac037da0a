set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in astep astep32; do
  BBVEC_LIB=$PWD/tools/variants/libbbvec_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_env_parity.py tests/test_gpu_full_parity.py tests/test_gpu_rollout.py tests/test_gpu_solver_stress.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/sa_pytest_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/sa_pytest_$v.log)"; [ $rc -eq 0 ] || { tail -20 gpurun_out/sa_pytest_$v.log; exit $rc; }
done
for r in 1 2; do for v in main astep astep32; do
  lib=$PWD/tools/variants/libbbvec_$v.so; [ $v = main ] && lib=$PWD/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
  BBVEC_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --mode step --steps 2000 --warmup 100 > gpurun_out/sa_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sa_${v}_$r.json'));print('$v', $r, '%.3e'%d['value'], d['roofline']['kernel_avg_ms'])"
done; done
for r in 1 2; do for v in main sync; do
  lib=$PWD/tools/variants/libbbvec_$v.so; [ $v = main ] && lib=$PWD/block-blast-ai---reinforcement-learning-agent_amd/libbbvec.so
  BBVEC_LIB=$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --warmup 5 > gpurun_out/sr_${v}_$r.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sr_${v}_$r.json'));print('roll $v', $r, '%.3e'%d['value'])"
done; done
