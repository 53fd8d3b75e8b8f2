#!/bin/bash
# GPU suite: parity tests, smoke, the default bench line (verified), optional
# rocprofv3 kernel stats of the bench.  Every GPU step has its own limit; the
# first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-suite}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.json; exit 1; }
cat $O/bench.json
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c4share_lanes1 --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr > $O/prof_c4share_lanes1.log 2>&1
  find $O/prof -name "*stats*"
fi
