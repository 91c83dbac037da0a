#!/bin/bash
# Diagnostics: pure-torch MLP graph replay, torch's bias reductions against GEMV bias gradients; then the agent's
# graphed fp32 step with the product's LinearF32Function (NaN canary).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for e in "keep" "keep mv"; do
  echo "== $e"
  timeout -k 10 200 python -u tools/diag_graph_reduce.py 100 $e 2> gpurun_out/dgr.err || { tail -3 gpurun_out/dgr.err; exit 1; }
done
timeout -k 10 300 python -u tools/diag_graph_grad.py none 100 > gpurun_out/dgg_fix.json 2> gpurun_out/dgg_fix.err || { tail -5 gpurun_out/dgg_fix.err; exit 1; }
echo "[agent, product fix] steps with a flagged gradient: $(grep -c '"param"' gpurun_out/dgg_fix.json)"
timeout -k 10 300 python -u tools/diag_graph_grad.py graphed 100 > gpurun_out/dgg_fix2.json 2> gpurun_out/dgg_fix2.err || { tail -5 gpurun_out/dgg_fix2.err; exit 1; }
echo "[agent after a graphed agent, product fix] steps with a flagged gradient: $(grep -c '"param"' gpurun_out/dgg_fix2.json)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_agent.py tests/test_gpu_train.py tests/test_gpu_network_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/fix_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/fix_pytest.log)"; exit $rc
