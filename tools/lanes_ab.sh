#!/bin/bash
# The C4 share at several (hardware queues, engine lanes) settings, alternating
# processes on one box (DQ_BENCH_HW_QUEUES: bench.py sets GPU_MAX_HW_QUEUES from
# it before HIP starts).   bash tools/lanes_ab.sh TAG ROUNDS
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
B="bench.py --no-c3 --no-c2 --no-c5 --no-rowtile --no-bgr --no-weighted --no-timing --no-cpu-baseline --steps 20 --warmup 10"
for i in $(seq 1 $2); do
  for cfg in 8:4 12:4 12:5 12:6 16:8; do
    q=${cfg%%:*}; l=${cfg##*:}
    DQ_BENCH_HW_QUEUES=$q timeout -k 10 200 python3 -u $B --lanes $l > $O/q${q}_l${l}_$i.json 2> $O/q${q}_l${l}_$i.err
    echo "q=$q lanes=$l $(python3 -c "import json,sys; d=[json.loads(x) for x in open(sys.argv[1]) if x.startswith('{')][-1]; print(d['config']['gpu_max_hw_queues'], d['ms_per_step'], d['verified']['ok'])" $O/q${q}_l${l}_$i.json)"
  done
done
