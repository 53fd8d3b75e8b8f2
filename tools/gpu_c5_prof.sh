set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/c5prof; mkdir -p $O
#timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
#tail -2 $O/pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/ns8 -o run -- python3 -u tools/c5_shards.py 8 4 2> $O/ns8.txt
tail -2 $O/ns8.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/ns1 -o run -- python3 -u tools/c5_shards.py 1 4 2> $O/ns1.txt
tail -2 $O/ns1.txt
