set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${C5AB_TAG:-c5ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_atsize.py tests/test_gpu_handoff.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  DQ_HIP_LIB=$(pwd)/ab_base.so timeout -k 10 200 python3 -u tools/c5_shards.py 8 4 2> $O/base8_$i.txt; tail -3 $O/base8_$i.txt | sed 's/^/base /'
  timeout -k 10 200 python3 -u tools/c5_shards.py 8 4 2> $O/new8_$i.txt; tail -3 $O/new8_$i.txt | sed 's/^/new /'
done
timeout -k 10 200 python3 -u tools/c5_shards.py 1 4 2> $O/new1.txt; tail -3 $O/new1.txt | sed 's/^/new /'
