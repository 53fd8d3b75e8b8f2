#!/bin/bash
# The round's closing evidence from ONE tree on one box: the GPU test suite,
# smoke(), a C3 device timeline (rocprofv3 kernel trace of tools/c3_trace.py
# + the host phase trace) and the default bench line.
#   bash tools/gpu_final.sh TAG        (outputs under gpurun_out/TAG)
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
export DQ_HIP_DIE_LOG=$O/die.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
DQ_HIP_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/c3prof -o run -- python3 -u tools/c3_trace.py 20 > $O/c3_calls.txt 2> $O/c3_host_trace.txt || { tail -5 $O/c3_host_trace.txt; exit 1; }
python3 tools/timeline.py $O/c3prof 130 > $O/timeline_c3.txt
tail -1 $O/c3_calls.txt
timeout -k 10 900 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -c 600 $O/bench_default.json
echo final done
