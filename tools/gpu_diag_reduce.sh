#!/bin/bash
# Diagnostics: torch reductions under graph replay (tools/diag_graph_reduce.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for m in plain zero keep; do
  timeout -k 10 200 python -u tools/diag_graph_reduce.py 200 $m 2> gpurun_out/dgr_$m.err || { tail -5 gpurun_out/dgr_$m.err; exit 1; }
done
