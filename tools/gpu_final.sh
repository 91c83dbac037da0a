#!/bin/bash
# Round-end evidence in one GPU call: smoke(), the whole -m gpu suite, then the
# default bench line + rocprofv3 kernel stats + PMC traffic (tools/gpu_profile.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_profile.sh "$TAG"
ARGS="--mode step --steps 2000 --warmup 100" PMC_ARGS="--kernels step_fused_kernel --steps-per-launch 1" bash tools/gpu_profile.sh "${TAG}_step"
