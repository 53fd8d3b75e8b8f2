#!/bin/bash
# Engine-lane sweep of the default bench (development tool): lanes 1..4, each
# twice, and 3 / 4 lanes with 8 hardware queues.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
run() { echo "$*: $(env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-rowtile --no-c3 --no-bgr --no-timing --no-verify --steps 20 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["config"]["engine_lanes"])')"; }
for rep in 1 2; do
  for L in 1 2 3 4; do run DQ_HIP_LANES=$L || exit 1; done
done
run DQ_HIP_LANES=3 GPU_MAX_HW_QUEUES=8 || exit 1
run DQ_HIP_LANES=4 GPU_MAX_HW_QUEUES=8 || exit 1
