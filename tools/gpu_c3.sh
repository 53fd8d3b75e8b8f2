#!/bin/bash
# C3 latency anatomy on the GPU box: host-side round trace and kernel timeline.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c3}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 120 python -u tools/c3_trace.py 20 > $O/c3.txt 2>&1
cat $O/c3.txt
DQ_HIP_TRACE=2 timeout -k 10 120 python -u tools/c3_trace.py 3 > $O/c3_trace.txt 2>&1
tail -30 $O/c3_trace.txt
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace -d $O/prof -o c3 --output-format csv -- python3 $R/tools/c3_trace.py 3 > $O/prof_c3.log 2>&1
find $O/prof -name "*kernel_trace*"
