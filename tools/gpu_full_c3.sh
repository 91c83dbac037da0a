set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/full_pytest.log; [ $rc -eq 0 ] || { grep -m3 -A25 "^E  \|Error" gpurun_out/full_pytest.log | head -60; exit $rc; }
for ac in bf16 none; do
  timeout -k 10 400 python tools/bench_ppo.py --envs 65536 --update-steps 200 --autocast $ac > gpurun_out/c3_${ac}.json 2> gpurun_out/c3_${ac}.err || { tail -5 gpurun_out/c3_${ac}.err; exit 1; }
  cat gpurun_out/c3_${ac}.json
done
