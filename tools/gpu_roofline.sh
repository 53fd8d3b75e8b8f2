#!/bin/bash
# The bench line and its rocprofv3 kernel statistics from ONE command: the
# C4 per-GPU share leg only, one engine lane everywhere (so every launch in
# the trace ran un-overlapped, like the bench's HIP-event roofline region),
# under `rocprofv3 --kernel-trace --stats`.  The dominant kernel's average
# duration in the stats must agree with the line's roofline.avg_launch_us.
#   bash tools/gpu_roofline.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- \
  python3 -u bench.py --lanes 1 --no-c3 --no-c2 --no-c5 --no-rowtile --no-bgr --no-cpu-baseline \
  > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
python3 tools/roofline_check.py $O/bench_prof.json $O/prof > $O/roofline_check.txt
cat $O/roofline_check.txt
