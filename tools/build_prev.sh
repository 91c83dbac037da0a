#!/bin/bash
# Build libbbvec.so from a git revision (default HEAD) into tools/variants/libbbvec_<name>.so with the
# working tree's shipped sources list and flags (runtime/build.py): the baseline arm of an A/B against
# the working tree (tools/gpu_ab.sh VARIANTS="prev main").
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=${1:-HEAD}
T=$(mktemp -d)
git -C "$R" archive "$REV" include block-blast-ai---reinforcement-learning-agent_amd/csrc | tar -x -C "$T"
mkdir -p "$R/tools/variants"
python3 - "$R" "$T" "${2:-prev}" <<'PY'
import os, subprocess, sys
R, T, name = sys.argv[1:4]
sys.path.insert(0, os.path.join(R, "block-blast-ai---reinforcement-learning-agent_amd"))
from runtime.build import HIPCC_FLAGS, SOURCES
C = os.path.join(T, "block-blast-ai---reinforcement-learning-agent_amd", "csrc")
srcs = [os.path.join(C, s) for s in SOURCES if os.path.exists(os.path.join(C, s))]
subprocess.run(["/opt/rocm/bin/hipcc", *HIPCC_FLAGS, f"-I{os.path.join(T, 'include')}", *srcs, "-o",
                os.path.join(R, "tools", "variants", f"libbbvec_{name}.so")], check=True)
PY
rm -rf "$T"
echo "$R/tools/variants/libbbvec_${2:-prev}.so ($REV)"
