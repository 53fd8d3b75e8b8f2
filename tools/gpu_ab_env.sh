#!/bin/bash
# A/B of one engine environment knob on the bench's C4-share, C3 and C2 legs
# (alternating runs, each with its own time limit; the first failure ends
# the call).    bash tools/gpu_ab_env.sh TAG "VAR=a" "VAR=b" [rounds]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
for i in $(seq 1 ${4:-2}); do
  for e in "$2" "$3"; do
    env $e timeout -k 10 200 python3 -u bench.py --no-c5 --no-rowtile --no-bgr --no-cpu-baseline --no-timing \
      > $O/ab_${i}_${e//=/_}.json 2> $O/ab_${i}_${e//=/_}.err || { tail -20 $O/ab_${i}_${e//=/_}.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/ab_${i}_${e//=/_}.json')); t=d['detail']
print('$e', 'c4share', d['ms_per_step'], 'c3', t['c3']['ms_per_frame'], 'c2', t['c2']['ms_per_frame'], 'ok', d['verified']['ok'], t['c3']['verified'], t['c2']['verified'])"
  done
done
