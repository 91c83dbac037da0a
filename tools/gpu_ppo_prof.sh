#!/bin/bash
# rocprofv3 kernel stats of the config-3 update step (bf16 autocast and fp32)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
for ac in ${ACS:-bf16 none}; do
  cd /tmp || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ppo_$ac" -o run --output-format csv -- python "$R/tools/bench_ppo.py" --envs 8192 --update-steps 60 --autocast $ac > "$R/gpurun_out/ppo_$ac.log" 2>&1 || { tail -20 "$R/gpurun_out/ppo_$ac.log"; exit 1; }
  tail -1 "$R/gpurun_out/ppo_$ac.log"
  f=$(find "$R/gpurun_out/ppo_$ac" -name "*kernel_stats.csv" | head -1); cp "$f" "$R/gpurun_out/ppo_${ac}_kernel_stats.csv"
  python3 - "$R/gpurun_out/ppo_${ac}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", round(tot / 1e6, 1), "kernels", len(rows))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
    print(f'{float(r["Percentage"]):6.2f}% {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f}us  {r["Name"][:110]}')
PY
done
