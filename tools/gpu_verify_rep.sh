#!/bin/bash
# Repeated verified bench runs (development tool): lanes 1 and default, plain
# and under rocprofv3 --kernel-trace, reporting the per-frame verification.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-vrep}
mkdir -p $O
cd $R
v() { python3 -c "
import json,sys
for l in open('$1'):
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print('$2', d.get('verified',{}).get('ok') if 'error' not in d else 'FAIL %s' % d.get('per_frame_rank0')); break
"; }
for i in 1 2 3; do
  timeout -k 10 120 python3 bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr > $O/l1_$i.json 2>/dev/null; v $O/l1_$i.json "lanes1 run$i"
done
cd /tmp
for i in 1 2; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof$i -o p --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr > $O/prof$i.log 2>&1; v $O/prof$i.log "rocprof lanes1 run$i"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof3 -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr > $O/prof3.log 2>&1; v $O/prof3.log "rocprof lanes3"
exit 0
