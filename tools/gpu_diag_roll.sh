#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in ${V:-diag3}; do
BBVEC_LIB=tools/variants/libbbvec_${v}.so timeout -k 10 300 python tools/diag_rollout.py > gpurun_out/diag_roll_$v.json 2> gpurun_out/diag_roll.err || { tail -20 gpurun_out/diag_roll.err; exit 1; }
python - gpurun_out/diag_roll_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))[-1]
print(sys.argv[2], d["cyc_per_wave_step"], d.get("multi_search_per_wave_step"), "max/mean", round(d["max_wave_total"] / d["mean_wave_total"], 3),
      "parked/wave-step", d["searches_per_wave_step"], "cyc/search", d["cyc_per_search"])
PY
done
