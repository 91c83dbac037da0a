set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for g in "" "--graph-rollout"; do
  for n in 65536 131072; do
    timeout -k 10 400 python tools/bench_ppo.py --envs $n --autocast bf16 --update-steps 50 $g > gpurun_out/c5_${n}${g}.json 2> gpurun_out/c5_${n}${g}.err || { tail -20 gpurun_out/c5_${n}${g}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/c5_${n}${g}.json'));print($n, '$g', d['rollout_s'], d['rollout_env_steps_per_s'], d['update_step_ms'], d['ppo_env_steps_per_s'])"
  done
done
