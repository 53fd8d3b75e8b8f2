#!/bin/bash
# GPU suite, then the bench's share step, C5 and C4 row-tile legs (no C3 /
# C2 / BGR24 / weighted legs) with and without DQ_HIP_TUNE settings,
# alternating processes on one box.   bash tools/gpu_tune_ab.sh TAG ROUNDS TUNE...
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
ROUNDS=$2
shift 2
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
B="bench.py --no-c3 --no-c2 --no-bgr --no-weighted --no-cpu-baseline --no-timing"
K='import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); t=d["detail"]; r=t.get("c4_rowtile",{}); c=t.get("c5",{}); print("share", d["ms_per_step"], d["verified"]["ok"], "c5", c.get("ms_per_tile"), c.get("verified"), "rowtile", r.get("ms_per_step"), r.get("verified"))'
for i in $(seq 1 $ROUNDS); do
  for t in tree "$@"; do
    if [ "$t" = tree ]; then unset DQ_HIP_TUNE; else export DQ_HIP_TUNE=$t; fi
    timeout -k 10 400 python3 -u $B > $O/${t}_$i.json 2> $O/${t}_$i.err
    echo "$t $(python3 -c "$K" $O/${t}_$i.json)"
  done
done
unset DQ_HIP_TUNE
echo tune ab done
