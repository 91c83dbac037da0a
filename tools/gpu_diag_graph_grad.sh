#!/bin/bash
# Diagnostics: tools/diag_graph_grad.py (NaN canary, lr-0 eager twin), 100 steps per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for v in "none 100" "none 100 mvlinear" "none 100" "none 100 mvlinear"; do
  i=$((i+1))
  timeout -k 10 300 python -u tools/diag_graph_grad.py $v > gpurun_out/dgg_v$i.json 2> gpurun_out/dgg_v$i.err || { tail -5 gpurun_out/dgg_v$i.err; exit 1; }
  echo "[$v] steps with a flagged gradient: $(grep -c '"param"' gpurun_out/dgg_v$i.json); first: $(grep -m1 -o '"step": [0-9]*, "bad": \[{"param": "[^"]*"' gpurun_out/dgg_v$i.json)"
done
