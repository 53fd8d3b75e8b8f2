#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (C3 single + 8-frame batch),
# rocprofv3 kernel-trace stats of the bench.  Every GPU step has its own limit;
# the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log
timeout -k 10 240 python -u bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
timeout -k 10 240 python -u bench.py --frames 8 --no-cpu-baseline > $O/bench_f8.json 2> $O/bench_f8.err
cat $O/bench_f8.json
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_c3.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o c3f8 --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --frames 8 --no-cpu-baseline > $O/prof_c3f8.log 2>&1
find $O/prof -name "*stats*" | head
