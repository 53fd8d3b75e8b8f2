set -e -o pipefail
O=gpurun_out/lanes; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
tail -1 $O/pytest.log
for L in 1 2 3 4; do
  DQ_HIP_LANES=$L timeout -k 10 120 python bench.py --no-cpu-baseline --no-timing --no-c3 --steps 20 > $O/b$L.json
  python3 -c "import json; d=json.load(open('$O/b$L.json')); print('lanes=$L', d['value'], d['ms_per_step'])"
done
DQ_HIP_LANES=2 timeout -k 10 120 python bench.py --no-cpu-baseline --no-timing --no-c3 --frames 16 --steps 10 > $O/f16.json
python3 -c "import json; d=json.load(open('$O/f16.json')); print('f16 lanes=2', d['value'], d['ms_per_step'])"
DQ_HIP_LANES=4 timeout -k 10 120 python bench.py --no-cpu-baseline --no-timing --no-c3 --frames 16 --steps 10 > $O/f16b.json
python3 -c "import json; d=json.load(open('$O/f16b.json')); print('f16 lanes=4', d['value'], d['ms_per_step'])"
