set -e -o pipefail
O=gpurun_out/sweep1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for cfg in "" "DQ_HIP_TILES=2048" "DQ_HIP_TILE_MAX=16384" "DQ_HIP_TILE_MAX=32768" "DQ_HIP_TILES=2048 DQ_HIP_TILE_MAX=16384"; do
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-timing --steps 10 > $O/b.json
  python3 -c "import json,sys; d=json.load(open('$O/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['detail']['c3'])"
done
