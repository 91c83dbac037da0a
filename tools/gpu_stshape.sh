#!/bin/bash
# bb_step single-step instantiation shapes (envs per wave, workgroup size): full-size parity, then interleaved
# step-mode bench repeats, then the env parity suites with the shipped build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/st; export TMPDIR=/tmp
V=${VARIANTS:-"main st16 st8 st32b256 st16b256 st8b256 st16b128"}
VARIANTS="$V" PARITY=1 REPS=0 bash tools/gpu_ab.sh st/p || exit 1
VARIANTS="$V" PARITY=0 REPS=${REPS:-2} ARGS="--mode step --steps 4000 --warmup 200" bash tools/gpu_ab.sh st/step || exit 1
