set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=block-blast-ai---reinforcement-learning-agent_amd
for E in 4 8 16 32; do
  lib=$P/libbbvec_e$E.so; [ $E = 8 ] && lib=$P/libbbvec.so
  cd /tmp && BBVEC_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/esc_e$E" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --steps 100 --warmup 10 > "$GRAFT_REPO_ROOT/gpurun_out/esc_e$E.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"
  f=$(find gpurun_out/esc_e$E -name "*kernel_stats.csv" | head -1)
  echo "E=$E"; grep -E "escalate|step_kernel" "$f" | cut -d, -f1,2,4,6,7 | sed 's/(bb::EnvDev[^"]*//'
done
