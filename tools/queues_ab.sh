#!/bin/bash
# The share (and C3) at 8 vs 12 hardware queues, 4 lanes, alternating processes
# (DQ_BENCH_HW_QUEUES: bench.py sets GPU_MAX_HW_QUEUES from it before HIP starts).
#   bash tools/queues_ab.sh TAG ROUNDS
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
B="bench.py --no-c2 --no-c5 --no-rowtile --no-bgr --no-weighted --no-timing --no-cpu-baseline --steps 30 --warmup 10"
for i in $(seq 1 $2); do
  for q in 8 12; do
    DQ_BENCH_HW_QUEUES=$q timeout -k 10 200 python3 -u $B > $O/q${q}_$i.json 2> $O/q${q}_$i.err
    echo "q=$q $(python3 -c "import json,sys; d=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][-1]; print(d['config']['gpu_max_hw_queues'], d['ms_per_step'], d['detail']['c3']['ms_per_frame'], d['verified']['ok'])" $O/q${q}_$i.json)"
  done
done
