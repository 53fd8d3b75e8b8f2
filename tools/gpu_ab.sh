#!/bin/bash
# Interleaved A/B of the default bench line over library variants
# (tools/build_variant.sh): bash tools/gpu_ab.sh TAG REPS NAME [NAME ...]
# ("default" = the in-tree library).  No CPU baseline, no verification.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; REPS=$2; shift 2
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for r in $(seq 1 $REPS); do
  for v in "$@"; do
    if [ "$v" = default ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/clusteringsegmentation-1_amd/variants/$v.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-rowtile --steps 20 --warmup 10 > $O/r${r}_$v.json 2> $O/r${r}_$v.err
    python3 -c "
import json; d=json.load(open('$O/r${r}_$v.json')); k=d['detail']['kernels']
print('rep $r %-8s %.0f Mpix/s %.3f ms/step c3 %.3f ms  partsplit %.1f us map %.1f us' % ('$v', d['value'], d['ms_per_step'], d['detail']['c3']['ms_per_frame'], k['partition']['ms']*1e3/k['partition']['launches'], k['map']['ms']*1e3/k['map']['launches']))"
  done
done
