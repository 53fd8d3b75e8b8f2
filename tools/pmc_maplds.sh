#!/bin/bash
# Counters of map_lds_kernel inside a short one-lane bench run (two passes).
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-pmcmap}
mkdir -p $O
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-timing --no-c3 --no-rowtile --no-bgr --no-verify --lanes 1"
K="--kernel-include-regex map_lds"
cd /tmp
timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o p -- python3 $R/bench.py $ARGS > $O/p1.log 2>&1
timeout -s KILL 90 rocprofv3 $K --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM --output-format csv -d $O/p2 -o p -- python3 $R/bench.py $ARGS > $O/p2.log 2>&1
python3 - "$O" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(acc):
    print("%-24s %16.0f  (%d rows)" % (k, acc[k], n[k]))
PY
