set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/bh; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_block_hist.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python -u tools/bench_blockhist.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o bh --output-format csv -- python3 $R/tools/bench_blockhist.py --cpu 0 > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats*" -exec cat {} \;
