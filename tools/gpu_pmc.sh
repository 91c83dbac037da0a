#!/bin/bash
# Two PMC passes (FETCH_SIZE, WRITE_SIZE) over the default bench, kernel-trace only.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
R="$GRAFT_REPO_ROOT"
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_fetch" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 50 --warmup 10 > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_fetch.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_write" -o run --output-format csv -- python "$R/bench.py" --no-cpu-baseline --steps 50 --warmup 10 > "$R/gpurun_out/${TAG}_write.log" 2>&1 || { tail -20 "$R/gpurun_out/${TAG}_write.log"; exit 1; }
python "$R/tools/pmc_traffic.py" "$R/gpurun_out/${TAG}_fetch" "$R/gpurun_out/${TAG}_write" --envs 65536 --out "$R/gpurun_out/${TAG}_traffic.json"
