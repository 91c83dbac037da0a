#!/bin/bash
# Per-kernel HBM bytes of the bf16 update step: a plain kernel trace and two separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) over tools/prof_update.py, summarised by tools/pmc_update.py.  usage: TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; TAG=${1:-upmc}; A="--batch 2048 --steps 10 --warm 5 ${PU_ARGS:-}"
cd /tmp || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/${TAG}_kt" -o run --output-format csv -- python3 "$R/tools/prof_update.py" $A > "$R/gpurun_out/${TAG}_kt.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_kt.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_fetch" -o run --output-format csv -- python3 "$R/tools/prof_update.py" $A > "$R/gpurun_out/${TAG}_fetch.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_fetch.log"; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/${TAG}_write" -o run --output-format csv -- python3 "$R/tools/prof_update.py" $A > "$R/gpurun_out/${TAG}_write.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_write.log"; exit 1; }
python3 "$R/tools/pmc_update.py" "$R/gpurun_out/${TAG}_kt" "$R/gpurun_out/${TAG}_fetch" "$R/gpurun_out/${TAG}_write" --out "$R/gpurun_out/${TAG}_update_pmc.txt" | head -40
