#!/bin/bash
# Round profile set for the default bench: full bench line (with CPU baseline),
# rocprofv3 kernel stats, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; TAG=${1:-prof}; ARGS=${ARGS:-"--steps 1280 --warmup 128"}
timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_kt" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline $ARGS > "$R/gpurun_out/${TAG}_kt.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_kt.log"; exit 1; }
f=$(find "$R/gpurun_out/${TAG}_kt" -name "*kernel_stats.csv" | head -1); cp "$f" "$R/gpurun_out/${TAG}_kernel_stats.csv"
cut -d, -f1-8 "$f" | grep "bb::" | cut -c1-60,200-400
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_fetch" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline $ARGS > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_write" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline $ARGS > "$R/gpurun_out/${TAG}_write.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_write.log"; exit 1; }
python "$R/tools/pmc_traffic.py" "$R/gpurun_out/${TAG}_fetch" "$R/gpurun_out/${TAG}_write" --envs 65536 ${PMC_ARGS:---kernels rollout_async_kernel --steps-per-launch 128} --out "$R/gpurun_out/${TAG}_pmc.json"
