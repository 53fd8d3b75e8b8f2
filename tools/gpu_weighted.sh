#!/bin/bash
# The weighted path on C3's frame: GPU tests of the path, timed calls, and a
# rocprofv3 kernel trace + stats of the same script.   bash tools/gpu_weighted.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q -k "weighted or varpart or cut_bits" --timeout 240 --timeout-method thread > $O/pytest_weighted.txt 2>&1 || { tail -30 $O/pytest_weighted.txt; exit 1; }
tail -1 $O/pytest_weighted.txt
timeout -k 10 300 python3 -u tools/weighted_c3.py 10 > $O/weighted_c3.json 2> $O/weighted_c3.err || { tail -20 $O/weighted_c3.err; exit 1; }
cat $O/weighted_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- python3 -u tools/weighted_c3.py 5 > $O/weighted_prof.json 2> $O/weighted_prof.err || { tail -20 $O/weighted_prof.err; exit 1; }
echo weighted done
