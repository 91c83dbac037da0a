#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=r06a
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_ppo_update_oracle.py tests/test_gpu_linear_tail.py tests/test_gpu_ppo_kernels.py tests/test_gpu_full_size.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 180 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/${TAG}_pu_$r.json 2> gpurun_out/${TAG}_pu_$r.err || { tail -5 gpurun_out/${TAG}_pu_$r.err; exit 1; }
tail -1 gpurun_out/${TAG}_pu_$r.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
