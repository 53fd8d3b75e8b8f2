#!/bin/bash
# GPU suite on the tree, then the latency A/B of tunings (tools/ab.sh) and a
# C3 trace.   bash tools/gpu_ab_c3.sh TAG CALLS ROUNDS TUNE...
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
T=$1; C=$2; N=$3
shift 3
export DQ_HIP_DIE_LOG=$O/die.txt
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
args=""
for t in "$@"; do args="$args tree:$t"; done
bash tools/ab.sh $T/ab $C $N tree $args
DQ_HIP_TRACE=1 timeout -k 10 300 python3 -u tools/c3_trace.py 10 > $O/c3_calls.txt 2> $O/c3_host.txt
tail -1 $O/c3_calls.txt
echo abc3 done
