#!/bin/bash
# C3 / C2 single-frame latency under engine environment settings (one bench
# process per setting, C3 and C2 legs only).
#   bash tools/gpu_c3_sweep.sh TAG "VAR=a VAR2=b" "VAR=c" ...
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
shift
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 150 python3 -u bench.py --frames 8 --steps 20 --warmup 5 --no-c5 --no-rowtile --no-bgr \
    --no-cpu-baseline --no-timing > $O/s$i.json 2> $O/s$i.err || { tail -20 $O/s$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/s$i.json')); t=d['detail']
print('$e', '| c4share', d['ms_per_step'], 'c3', t['c3']['ms_per_frame'], 'c2', t['c2']['ms_per_frame'], 'ok', d['verified']['ok'], t['c3']['verified'], t['c2']['verified'])"
done
