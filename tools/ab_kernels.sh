#!/bin/bash
# Per-kernel times (the bench's HIP-event region, one engine lane, 8 x 4K) of
# several library builds on one box, alternating processes.
#   bash tools/ab_kernels.sh TAG ROUNDS LIB[:TUNE]...   (LIB: a .so path, or "tree";
#   TUNE: a DQ_HIP_TUNE list for that run)
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
ROUNDS=$2
shift 2
mkdir -p $O
cd $R
B="bench.py --lanes 1 --no-c3 --no-c2 --no-c5 --no-rowtile --no-bgr --no-cpu-baseline --steps 20 --warmup 5"
K='import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1]); print(d["ms_per_step"], d["verified"]["ok"], {k:(v["launches"],round(v["ms"]*1e3/v["launches"],1)) for k,v in d["detail"]["kernels"].items()})'
for i in $(seq 1 $ROUNDS); do
  for L in "$@"; do
    lib=${L%%:*}
    tune=""
    [ "$lib" != "$L" ] && tune=${L#*:}
    t=$(basename $lib .so)${tune:+_$tune}
    t=${t//[=,]/_}
    if [ "$lib" = tree ]; then DQ_HIP_TUNE=$tune timeout -k 10 200 python3 -u $B > $O/${t}_$i.json
    else DQ_HIP_TUNE=$tune DQ_HIP_LIB=$R/$lib timeout -k 10 200 python3 -u $B > $O/${t}_$i.json; fi
    echo "$t $(python3 -c "$K" $O/${t}_$i.json)"
  done
done
