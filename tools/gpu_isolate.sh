#!/bin/bash
# The shard / loopback GPU tests (the order the arena check runs last in)
# under each given library build, in turn, stopping at the first failure.
#   bash tools/gpu_isolate.sh TAG LIB...      (LIB: a .so path, or "tree")
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
for L in "$@"; do
  t=$(basename $L .so)
  export DQ_HIP_DIE_LOG=$O/die_$t.txt
  if [ "$L" = tree ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/$L; fi
  timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rows.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_$t.txt 2>&1 || { tail -30 $O/pytest_$t.txt; exit 1; }
  echo "$t: $(tail -1 $O/pytest_$t.txt)"
done
