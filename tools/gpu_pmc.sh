#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc run per group: rocprofv3 does not
# split counters over passes) over the bench's 8 x 4K leg, one engine lane.
#   bash tools/gpu_pmc.sh TAG "CNT CNT ..." ["CNT ..." ...]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
B="bench.py --lanes 1 --no-c3 --no-c2 --no-c5 --no-rowtile --no-bgr --no-cpu-baseline --no-timing --steps 2 --warmup 1"
i=0
for G in "$@"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $G -f csv -d $O/p$i -o run -- python3 -u $B > $O/p$i.json 2> $O/p$i.err || { tail -5 $O/p$i.err; exit 1; }
done
python3 tools/pmc_table.py $O > $O/table.txt
echo pmc done
