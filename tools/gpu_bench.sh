#!/bin/bash
# Bench lines + rocprofv3 kernel stats for one tag (no tests).
#   default command (engine lanes overlap kernels) and the same command with
#   --lanes 1 (kernels un-overlapped: the profile the roofline object agrees with)
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
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c4share_lanes1 --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 > $O/prof_c4share_lanes1.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c4share --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 > $O/prof_c4share.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c5 --output-format csv -- python3 $R/bench.py --mode rows --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c5.log 2>&1
echo done
