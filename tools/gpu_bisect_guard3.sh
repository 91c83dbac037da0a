#!/bin/bash
# Diagnostics: does an unwritten-memory read (NaN-poisoned allocator) reproduce the Adam guard in train()?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for pz in nan graphed; do
  for md in eager graphs; do
    timeout -k 10 240 python -u tools/diag_guard.py $md $pz > gpurun_out/dg_${pz}_$md.json 2> gpurun_out/dg_${pz}_$md.err
    rc=$?; echo "$pz $md rc=$rc"; cut -c1-1500 gpurun_out/dg_${pz}_$md.json
    [ $rc -eq 0 ] || { tail -5 gpurun_out/dg_${pz}_$md.err; exit $rc; }
  done
done
