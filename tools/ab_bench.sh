#!/bin/bash
# The bench's share step and C4 row-tile leg (no C3/C2/C5/BGR legs) of several
# library builds on one box, alternating processes.
#   bash tools/ab_bench.sh TAG ROUNDS LIB...   (LIB: a .so path, or "tree")
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
ROUNDS=$2
shift 2
mkdir -p $O
cd $R
B="bench.py --no-c3 --no-c2 --no-c5 --no-bgr --no-cpu-baseline --no-timing"
K='import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); r=d["detail"].get("c4_rowtile",{}); print(d["ms_per_step"], d["verified"]["ok"], r.get("ms_per_step"), r.get("verified"), round(r.get("ms_per_step",0)/8/d["ms_per_step"],3))'
for i in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    t=$(basename $L .so)
    if [ "$L" = tree ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/$L; fi
    timeout -k 10 300 python3 -u $B > $O/${t}_$i.json 2> $O/${t}_$i.err
    echo "$t $(python3 -c "$K" $O/${t}_$i.json)"
  done
done
