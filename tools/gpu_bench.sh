#!/bin/bash
# Bench lines + rocprofv3 kernel stats for one tag (no tests).
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-bench}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 300 python -u bench.py --mode rows --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
cat $O/bench_c5.json
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c4share --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 > $O/prof_c4share.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 --output-format csv -- python3 $R/bench.py --frames 1 --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c3.log 2>&1
echo done
