#!/bin/bash
# Sharded-path check and timing: the shard / loopback / arena-check GPU tests
# first, then C5 with 1 and 8 virtual row shards under rocprofv3 kernel stats.
#   bash tools/gpu_shards.sh TAG
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
export DQ_HIP_DIE_LOG=$O/die.txt
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rows.py tests/test_gpu_loopback.py tests/test_gpu_atsize.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for ns in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/ns$ns -o run -- python3 -u tools/c5_shards.py $ns 4 2> $O/ns${ns}_calls.txt > /dev/null || { tail -5 $O/ns${ns}_calls.txt; exit 1; }
  tail -2 $O/ns${ns}_calls.txt
done
echo shards done
