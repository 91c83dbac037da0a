#!/bin/bash
# bb_optim.hip: its GPU tests, then an A/B of the config-3 optimizer step (bf16 autocast)
# with the fused clip+Adam / multi-tensor Linear casts / residual BatchNorm tail on and off (env flags).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-optab}
timeout -k 10 400 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_ppo_agent.py tests/test_gpu_conv.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-on off}; do
    case $v in
      on) fa=1; fc=1; rf=1;; off) fa=0; fc=0; rf=0;; adam) fa=1; fc=0; rf=0;; cast) fa=0; fc=1; rf=0;;
      nores) fa=1; fc=1; rf=0;;
    esac
    pm=1; ex=""; [ $v = noprep ] && { fa=1; fc=1; rf=1; pm=0; }
    [ $v = copyin ] && { fa=1; fc=1; rf=1; ex=--copy-inputs; }
    rg=1; [ $v = norg ] && { fa=1; fc=1; rf=1; rg=0; }
    BB_RES_GRAD_FUSED=$rg BB_FUSED_ADAM=$fa BB_FUSED_CASTS=$fc BB_RES_FUSED=$rf BB_PREP_MULTI=$pm timeout -k 10 200 python tools/bench_ppo.py --envs 8192 --update-steps 300 --autocast bf16 $ex > gpurun_out/${TAG}_${v}_$r.json 2>gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${v}_$r.json'));print('$v', $r, d['update_step_ms'])"
  done
done
