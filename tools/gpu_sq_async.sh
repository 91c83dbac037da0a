#!/bin/bash
# What binds rollout_async_kernel: SQ counters of the bench kernel (separate --pmc passes, kernel trace only),
# the per-wave-type time split of the diagnostic build (tools/diag_async.py, tools/variants/libbbvec_adiag.so),
# and the VALU issue microbenchmarks (tools/ubench/*, prebuilt on the CPU side).
# usage: tools/gpu_sq_async.sh TAG   (outputs under gpurun_out/TAG_*)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sqa}; R=$GRAFT_REPO_ROOT
ARGS=${ARGS:-"--steps 20 --warmup 10 --no-cpu-baseline"}
cd /tmp || exit 1
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/${TAG}_counters.txt" 2>&1 || true
i=0
for set in ${SETS:-SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_INST_ANY,SQ_WAIT_ANY,SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_LDS,SQ_INSTS_SMEM,SQ_INSTS_VMEM_WR,SQ_INSTS_VMEM_RD,SQ_BUSY_CYCLES,SQ_INSTS_BRANCH SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_MISC,SQ_INST_CYCLES_VMEM_WR,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_VMEM,SQ_INST_LEVEL_VMEM,GRBM_GUI_ACTIVE,GRBM_COUNT}; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc ${set//,/ } --kernel-trace -d "$R/gpurun_out/${TAG}_p$i" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/${TAG}_p$i.log" 2>&1 || { tail -5 "$R/gpurun_out/${TAG}_p$i.log"; echo "pass $i failed"; }
done
cd "$R" || exit 1
python3 tools/sq_summary.py gpurun_out "$TAG" rollout_async_kernel > gpurun_out/${TAG}_sq.txt; cat gpurun_out/${TAG}_sq.txt
if [ -z "$NODIAG" ] && [ -f tools/variants/libbbvec_adiag.so ]; then
  BBVEC_LIB=tools/variants/libbbvec_adiag.so timeout -k 10 120 python3 tools/diag_async.py > gpurun_out/${TAG}_diag.json 2> gpurun_out/${TAG}_diag.err || { tail -5 gpurun_out/${TAG}_diag.err; exit 1; }
  tail -20 gpurun_out/${TAG}_diag.json
fi
for b in ${UBENCH:-}; do
  [ -x $b ] && { timeout -k 10 60 $b > gpurun_out/${TAG}_$(basename $b).txt 2>&1 || exit 1; cat gpurun_out/${TAG}_$(basename $b).txt; }
done
exit 0
