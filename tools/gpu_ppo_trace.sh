#!/bin/bash
# steady-state kernel breakdown of the config-3 update step: kernel trace, last 40% of the run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; AC=${AC:-bf16}
cd /tmp || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace -d "$R/gpurun_out/ppot" -o run --output-format csv -- python "$R/tools/bench_ppo.py" --envs 8192 --update-steps 400 --autocast $AC > "$R/gpurun_out/ppot.log" 2>&1 || { tail -20 "$R/gpurun_out/ppot.log"; exit 1; }
f=$(find "$R/gpurun_out/ppot" -name "*kernel_trace.csv" | head -1)
python3 - "$f" "$R/gpurun_out/ppo_steady_${AC}.txt" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
cut = t0 + 0.6 * (t1 - t0)
sel = [r for r in rows if int(r["Start_Timestamp"]) >= cut]
span = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
acc = collections.defaultdict(lambda: [0, 0])
for r in sel:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    acc[r["Kernel_Name"]][0] += d
    acc[r["Kernel_Name"]][1] += 1
busy = sum(v[0] for v in acc.values())
lines = [f"window {span/1e6:.1f} ms, kernel busy {busy/1e6:.1f} ms ({100*busy/span:.1f}%), {len(sel)} kernels"]
for k, (d, c) in sorted(acc.items(), key=lambda kv: -kv[1][0])[:30]:
    lines.append(f"{100*d/busy:6.2f}% {c:7d} {d/c/1e3:8.1f}us  {k[:120]}")
open(sys.argv[2], "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
PY
rm -rf "$R/gpurun_out/ppot"
