#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
BBVEC_LIB=tools/variants/libbbvec_${V:-diag3}.so timeout -k 10 300 python tools/diag_rollout.py > gpurun_out/diag_roll.json 2> gpurun_out/diag_roll.err || { tail -20 gpurun_out/diag_roll.err; exit 1; }
cat gpurun_out/diag_roll.json
