#!/bin/bash
# Interleaved A/B of the default bench line over environment settings
# (development tool): bash tools/gpu_envab.sh TAG REPS "VAR=a" "VAR=b" ...
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; REPS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for r in $(seq 1 $REPS); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-rowtile --no-bgr --steps 20 --warmup 10 > $O/r${r}_$i.json 2> $O/r${r}_$i.err
    python3 -c "
import json; d=json.load(open('$O/r${r}_$i.json')); k=d['detail']['kernels']
print('rep $r %-28s %.0f Mpix/s %.3f ms/step c3 %.3f ms  partsplit %.1f us epi %d' % ('$v', d['value'], d['ms_per_step'], d['detail']['c3']['ms_per_frame'], k['partition']['ms']*1e3/k['partition']['launches'], k.get('epilogue',{}).get('launches',0)))"
  done
done
