#!/bin/bash
# One tuning build of libbbvec.so with extra -D flags (load with BBVEC_LIB=tools/variants/libbbvec_<name>.so).
#   tools/build_variant.sh <name> -DBB_ROLL_ENVS=32 ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/block-blast-ai---reinforcement-learning-agent_amd/csrc
name=$1; shift
mkdir -p $R/tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result \
  "$@" -I$R/include $C/bb_env.hip $C/bb_ppo.hip $C/bb_nn.hip $C/bb_loss.hip $C/bb_capi.cpp $C/bb_tables.cpp -o $R/tools/variants/libbbvec_$name.so
