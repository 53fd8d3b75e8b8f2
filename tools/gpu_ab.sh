#!/bin/bash
# GPU suite, then A/B timings of engine options (tools/ab_timing.py, one
# process per setting), then C2 / C3 device timelines of the default build.
#   bash tools/gpu_ab.sh TAG "ENV=.. ENV=.." "ENV=.." ...
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for setting in "$@"; do
  echo "[ab] $setting"
  env $setting timeout -k 10 150 python3 -u tools/ab_timing.py "$setting" 20 >> $O/ab.jsonl 2>> $O/ab.err \
    || { tail -20 $O/ab.err; exit 1; }
  tail -1 $O/ab.jsonl
done
for c in c3 c2; do
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/tl_$c -o run -- python3 -u tools/c2_trace.py $c 6 \
    > $O/tl_$c.log 2>&1 || { tail -20 $O/tl_$c.log; exit 1; }
  python3 tools/timeline.py $O/tl_$c 70 > $O/timeline_$c.txt
  tail -14 $O/timeline_$c.txt
done
