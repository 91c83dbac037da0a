#!/bin/bash
# Tuning builds of libbbvec.so with other escalation launch shapes (load with BBVEC_LIB=...).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/block-blast-ai---reinforcement-learning-agent_amd/csrc
for v in "$@"; do
  blk=${v%_*}; grp=${v#*_}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-result \
    -DBB_ESC_BLOCK=$blk -DBB_ESC_GROUP=$grp -I$R/include $C/bb_env.hip $C/bb_ppo.hip $C/bb_capi.cpp $C/bb_tables.cpp \
    -o $R/tools/variants/libbbvec_$v.so &
done
wait
