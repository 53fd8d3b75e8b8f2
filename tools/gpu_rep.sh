#!/bin/bash
# Repeat the GPU test suite (nondeterminism hunt).  Continues after plain test
# failures (pytest rc 1), stops on anything else (timeout, crash).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-rep}
mkdir -p $O
cd $R
for i in 1 2 3; do
  for plan in 1 1 0; do
    DQ_HIP_PLAN=$plan timeout -k 10 300 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:randomly > $O/run_${i}_$plan.log 2>&1
    rc=$?
    echo "iter $i plan $plan rc $rc: $(tail -1 $O/run_${i}_$plan.log)"
    grep -E "^FAILED" $O/run_${i}_$plan.log | head -5
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
