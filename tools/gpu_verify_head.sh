set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${VTAG:-vhead}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rows.py tests/test_gpu_atsize.py tests/test_gpu_handoff.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/shard_first.log 2>&1 || { tail -30 $O/shard_first.log; exit 1; }
tail -1 $O/shard_first.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
