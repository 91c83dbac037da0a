#!/bin/bash
# Experiment: PyTorch TunableOp (hipBLASLt / rocBLAS solution search) on the bf16 optimizer step's GEMMs.
# Pass 1 tunes in-process (results -> gpurun_out/tunableop_results*.csv); pass 2 only reads that file.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 120 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/to_base_$r.json 2> gpurun_out/to_base_$r.err || { tail -5 gpurun_out/to_base_$r.err; exit 1; }
  echo "base $r $(cat gpurun_out/to_base_$r.json)"
done
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv \
  timeout -k 10 600 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/to_tune.json 2> gpurun_out/to_tune.err || { tail -5 gpurun_out/to_tune.err; exit 1; }
echo "tuning run $(cat gpurun_out/to_tune.json)"
ls -la gpurun_out/tunableop_results*.csv
for r in 1 2; do
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv \
    timeout -k 10 120 python tools/prof_update.py --batch 2048 --steps 200 > gpurun_out/to_tuned_$r.json 2> gpurun_out/to_tuned_$r.err || { tail -5 gpurun_out/to_tuned_$r.err; exit 1; }
  echo "tuned $r $(cat gpurun_out/to_tuned_$r.json)"
done
