#!/bin/bash
# A/B latency (tools/latency.py medians: C3, C2, the 8 x 4K batch) of several
# library builds / tunings on one box, alternating processes.
#   bash tools/ab.sh TAG CALLS ROUNDS LIB[:TUNE]...   (LIB: a .so path, or
#   "tree"; TUNE: a DQ_HIP_TUNE list for that run)
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
CALLS=$2
ROUNDS=$3
shift 3
mkdir -p $O
cd $R
K='import json,sys; d=json.loads(open(sys.argv[1]).read()); print({k:(v["median_ms"],v["p10"],v["p90"]) for k,v in d.items() if k!="env"})'
for i in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    lib=${L%%:*}
    tune=""
    [ "$lib" != "$L" ] && tune=${L#*:}
    t=$(basename $lib .so)${tune:+_$tune}
    t=${t//[=,]/_}
    if [ "$lib" = tree ]; then DQ_HIP_TUNE=$tune timeout -k 10 200 python3 -u tools/latency.py $CALLS > $O/${t}_$i.json
    else DQ_HIP_TUNE=$tune DQ_HIP_LIB=$R/$lib timeout -k 10 200 python3 -u tools/latency.py $CALLS > $O/${t}_$i.json; fi
    echo "$t $(python3 -c "$K" $O/${t}_$i.json)"
  done
done
