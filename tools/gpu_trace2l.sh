#!/bin/bash
# Kernel trace of the default (2-lane) bench, for tools/overlap.py (development tool).
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-trace2l}
mkdir -p $O
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o lanes2 -- python3 $R/bench.py --steps 5 --warmup 5 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr --no-timing > $O/prof.log 2>&1
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 $R/tools/overlap.py $f --span 3000 --show 80
