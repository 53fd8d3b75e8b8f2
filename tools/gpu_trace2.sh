#!/bin/bash
# Kernel trace of the default bench (2 lanes): stream overlap.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace2
mkdir -p $O
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace -d $O -o t --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3 --no-rowtile --no-timing --no-verify > $O/bench.log 2>&1
F=$(find $O -name "*kernel_trace.csv" | head -1)
python3 $R/tools/overlap.py $F --span 3000 --show 120
