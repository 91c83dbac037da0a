#!/bin/bash
# Round 3: update-oracle tests, rollout A/B (main vs early-draw variant), SQ counters
# of both, and the diag3 phase breakdown of the rollout kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03d}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ppo_update_oracle.py -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || exit $rc
VARIANTS="${VARIANTS:-main dearly}" PARITY=1 REPS=3 bash tools/gpu_ab.sh ${TAG}_ab || exit 1
VARIANTS="${VARIANTS:-main dearly}" bash tools/gpu_sq_ab.sh ${TAG}_sq || exit 1
BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_diag3.so T=128 timeout -k 10 200 python tools/diag_rollout.py > gpurun_out/${TAG}_diag3.json 2> gpurun_out/${TAG}_diag3.err || { tail -5 gpurun_out/${TAG}_diag3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_diag3.json')); print(json.dumps(d[-1]))"
