#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-s4}
b() { # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['value']/1e6,1), d['roofline']['kernel_avg_ms'])"
}
b def || exit 1
for v in ${VARIANTS:-128_16 64_8 64_16 128_32 64_32 128_4}; do b v$v BBVEC_LIB=$GRAFT_REPO_ROOT/tools/variants/libbbvec_$v.so || exit 1; done
b def2 || exit 1
