#!/bin/bash
# C4-share bench under lane counts, at the box's default hardware queues (one process each).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
run() { echo "$*: $(env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-rowtile --no-c3 --no-timing --steps 20 2>/dev/null | python -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d["value"], d["ms_per_step"], d["config"]["engine_lanes"], d["verified"]["ok"])')"; }
for rep in 1 2 3; do
  run DQ_HIP_LANES=1
  run DQ_HIP_LANES=2
  run DQ_HIP_LANES=3
  run DQ_HIP_LANES=4
done
