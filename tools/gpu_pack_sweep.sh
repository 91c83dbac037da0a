#!/bin/bash
# bb_step / rollout: the wave search's attempts per env in the first and later rounds (BB_PACK_FIRST /
# BB_PACK_NEXT, runtime knobs), interleaved repeats.   PF="8 4 2" PN="32" MODE=step bash tools/gpu_pack_sweep.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-pack}
if [ "${MODE:-step}" = step ]; then A="--mode step --steps 2000 --warmup 100"; else A="--steps 640 --warmup 64"; fi
for r in $(seq 1 ${REPS:-2}); do
  for pf in ${PF:-8 4 2}; do for pn in ${PN:-32}; do
    BB_PACK_FIRST=$pf BB_PACK_NEXT=$pn timeout -k 10 120 python bench.py --no-cpu-baseline $A > gpurun_out/${TAG}_${pf}_${pn}_$r.json 2> gpurun_out/${TAG}_${pf}_${pn}_$r.err || { tail -5 gpurun_out/${TAG}_${pf}_${pn}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${pf}_${pn}_$r.json'));print('pf=$pf pn=$pn', $r, '%.3e'%d['value'], d['roofline']['kernel_avg_ms'])"
  done; done
done
