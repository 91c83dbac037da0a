set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS=60 timeout -k 10 300 python tools/diag_solver.py > gpurun_out/diag_solver.json 2> gpurun_out/diag_solver.err || { tail gpurun_out/diag_solver.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/diag_solver.json'))
print({k:d[k] for k in ('searches','cycles','attempts','passes','frac_any_slow','totals_cycles')})
print(d['per_step(t,n,max_cycles)'])"
