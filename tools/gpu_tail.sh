#!/bin/bash
# bb_step (T = 1) tail diagnostics on the diag3 build (tools/diag_step_tail.py).
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-tail}
BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_diag3.so timeout -k 10 300 python -u tools/diag_step_tail.py > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -5 gpurun_out/${TAG}.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}.json')); print(json.dumps(d['mean_over_calls']))"
