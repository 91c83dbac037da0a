set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=${OUT:-prof}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/$OUT" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 200 --warmup 20 > "$GRAFT_REPO_ROOT/gpurun_out/$OUT.log" 2>&1 || exit $?
f=$(find "$GRAFT_REPO_ROOT/gpurun_out/$OUT" -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -12
