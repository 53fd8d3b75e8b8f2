#!/bin/bash
# Long run-to-run stress of the C4 batch call: plain over 1-3 lanes, then one
# lane under rocprofv3 --kernel-trace (the configuration of the one
# unreproduced failure).  First failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-stress_long}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/stress_c4.py 5000 1 2 3 > $O/plain.log 2>&1 || { tail -20 $O/plain.log; exit 1; }
tail -2 $O/plain.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/stress_prof -o st --output-format csv -- python3 $R/tools/stress_c4.py 2000 1 > $O/rocprof.log 2>&1 || { tail -20 $O/rocprof.log; exit 1; }
grep -E "^call .*lanes|^calls" $O/rocprof.log | tail -5
