#!/bin/bash
# Build libbbvec.so from a git revision (default HEAD) into tools/variants/libbbvec_prev.so,
# the baseline arm of an A/B against the working tree (tools/gpu_ab.sh VARIANTS="prev main").
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
T=$(mktemp -d)
git -C "$R" archive "$REV" include block-blast-ai---reinforcement-learning-agent_amd/csrc | tar -x -C "$T"
C=$T/block-blast-ai---reinforcement-learning-agent_amd/csrc
mkdir -p "$R/tools/variants"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result \
  -I"$T/include" $C/bb_env.hip $C/bb_ppo.hip $C/bb_nn.hip $C/bb_loss.hip $C/bb_capi.cpp $C/bb_tables.cpp \
  -o "$R/tools/variants/libbbvec_${2:-prev}.so"
rm -rf "$T"
echo "$R/tools/variants/libbbvec_${2:-prev}.so ($REV)"
