set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/stepkt" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --mode step --steps 400 --warmup 40 > "$R/gpurun_out/stepkt.log" 2>&1 || { tail -20 "$R/gpurun_out/stepkt.log"; exit 1; }
f=$(find "$R/gpurun_out/stepkt" -name "*kernel_stats.csv" | head -1); cp "$f" "$R/gpurun_out/step_kernel_stats.csv"
python - "$R/gpurun_out/step_kernel_stats.csv" <<'PY'
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:4]: print(r['Name'][:30], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
PY
