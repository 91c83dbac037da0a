#!/bin/bash
# Diagnostics: tools/diag_graph_grad.py after each kind of earlier agent activity.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for pz in ${POISONS:-graphed_keep graphed_keep:noloss graphed_keep:adam0 none}; do
  i=$((i+1)); kind=${pz%%:*}; opt=${pz#*:}; [ "$opt" = "$pz" ] && opt=""
  envs=""; [ "$opt" = adam0 ] && envs="BB_FUSED_ADAM=0"
  env $envs timeout -k 10 240 python -u tools/diag_graph_grad.py $kind ${STEPS:-16} $opt > gpurun_out/dgg_$i.json 2> gpurun_out/dgg_$i.err
  rc=$?; echo "== $pz rc=$rc"
  grep -o '"step": [0-9]*\|{"param": "[^"]*", "rel": [0-9.e+-]*, "n_diff": [0-9]*' gpurun_out/dgg_$i.json | tr '\n' ' ' | sed 's/"step"/\n"step"/g' | cut -c1-400
  echo
  [ $rc -eq 0 ] || { tail -5 gpurun_out/dgg_$i.err; exit $rc; }
done
