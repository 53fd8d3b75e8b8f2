#!/bin/bash
# One GPU-box iteration: GPU parity suite, the default bench line, optional
# extra steps.  Every GPU step has its own time limit; the first failure ends
# the call (no retries).
#   bash tools/gpu_run.sh TAG [extra-step-script]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "[gpu_run] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo "[gpu_run] bench"
timeout -k 10 420 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err \
  || { tail -20 $O/bench.err; cat $O/bench.json; exit 1; }
python3 -c "
import json,sys; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'verified', d['verified']['ok'], 'frac', d['roofline']['frac'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])
print({k: v for k, v in d['detail'].items() if k in ('c3', 'c2', 'c5', 'c4_rowtile')})
"
if [ -n "$2" ]; then echo "[gpu_run] extra: $2"; bash $2 $O; fi
