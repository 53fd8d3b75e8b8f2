#!/bin/bash
# Repeat the verified one-lane bench (plain and under rocprofv3) to catch a
# rare wrong result (development tool); stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-race}
N=${2:-12}
mkdir -p $O
cd /tmp
for i in $(seq 1 $N); do
  timeout -k 10 120 rocprofv3 --kernel-trace -d $O/p$i -o p --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr --no-timing > $O/r$i.log 2>&1
  rc=$?
  if grep -q '"error"' $O/r$i.log; then echo "run $i FAILED"; grep '"error"' $O/r$i.log | cut -c1-900; exit 0; fi
  [ $rc -ne 0 ] && { echo "run $i rc=$rc"; tail -3 $O/r$i.log; exit 1; }
  rm -rf $O/p$i
  echo "run $i ok"
done
for i in $(seq 1 $N); do
  timeout -k 10 120 python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr --no-timing > $O/q$i.log 2>&1
  if grep -q '"error"' $O/q$i.log; then echo "plain run $i FAILED"; grep '"error"' $O/q$i.log | cut -c1-900; exit 0; fi
done
echo "plain runs ok"
