#!/bin/bash
# Instruction-mix counters of partsplit / pass kernels over a short bench run.
#   bash tools/pmc_valu.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmcv}
O=$R/gpurun_out/$TAG
mkdir -p $O
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-timing --no-c3 --lanes 1"
K="--kernel-include-regex (partsplit|pass_kernel|map_lds|build_cells)"
cd /tmp
timeout -s KILL 120 rocprofv3 $K --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/mix -o mix -- python3 $R/bench.py $ARGS > $O/mix.log 2>&1
python3 - "$O/mix" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    if r["Counter_Name"] == "SQ_WAVES": n[k] += 1
for k, c in acc.items():
    print(k, "dispatches", n[k], {x: "%.3g" % (v / max(n[k], 1)) for x, v in sorted(c.items())})
PY
