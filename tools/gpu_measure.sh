#!/bin/bash
# Measurements of the current tree on one GPU box (no test suite):
#   1. the default bench line (every leg, CPU baseline included);
#   2. the roofline pair (tools/gpu_roofline.sh: bench line + rocprofv3
#      stats of the same command);
#   3. device timelines of single-frame calls (C3, C2) under
#      rocprofv3 --kernel-trace (tools/timeline.py).
#   bash tools/gpu_measure.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
echo "[measure] bench (default)"
timeout -k 10 420 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'verified', d['verified']['ok'], 'frac', d['roofline']['frac'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])
print({k: v for k, v in d['detail'].items() if k in ('c3', 'c2', 'c5', 'c4_rowtile', 'bgr24_input')})
print('cpu', d.get('cpu_baseline'))
"
echo "[measure] roofline pair"
bash tools/gpu_roofline.sh $1/roof
for c in c3 c2; do
  echo "[measure] $c timeline"
  timeout -k 10 120 rocprofv3 --kernel-trace -f csv -d $O/tl_$c -o run -- python3 -u tools/c2_trace.py $c 6 \
    > $O/tl_$c.log 2>&1 || { tail -20 $O/tl_$c.log; exit 1; }
  python3 tools/timeline.py $O/tl_$c 70 > $O/timeline_$c.txt
  tail -16 $O/timeline_$c.txt
done
