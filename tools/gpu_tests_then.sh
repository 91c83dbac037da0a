#!/bin/bash
# Selected -m gpu test files (FILES), then each command in CMDS (';;'-separated, each under its own
# time limit, output to gpurun_out/TAG_cN.log).  One GPU call.  usage: FILES="..." CMDS="a;;b" tools/gpu_tests_then.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1
if [ -n "$FILES" ]; then
  timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/${TAG}_pytest.log | tail -3
  [ $rc -eq 0 ] || { grep -B5 -A30 "^E " gpurun_out/${TAG}_pytest.log | head -80; exit $rc; }
fi
i=0
IFS=$'\n'
for c in $(echo "$CMDS" | sed 's/;;/\n/g'); do
  i=$((i+1))
  echo "== c$i: $c"
  timeout -k 10 ${CMD_TIMEOUT:-300} bash -c "$c" > gpurun_out/${TAG}_c$i.log 2>&1
  rc=$?; tail -${TAIL:-5} gpurun_out/${TAG}_c$i.log
  [ $rc -eq 0 ] || { echo "c$i rc=$rc"; exit $rc; }
done
exit 0
