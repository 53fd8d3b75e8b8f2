#!/bin/bash
# The one-launch small weighted path: its GPU tests and the weighted tests of
# the suite (both paths), then the region-size latencies beside the reference.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-wsmall}
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_wsmall.py tests/test_gpu_parity.py -k "wsmall or weighted" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 300 python3 -u tools/weighted_regions.py > $O/regions.jsonl 2> $O/regions.err || { tail -5 $O/regions.err; exit 1; }
cat $O/regions.jsonl
