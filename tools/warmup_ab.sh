set -e -o pipefail
O=gpurun_out/wu; mkdir -p $O
for r in 1 2 3; do
  for w in 3 10; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --no-timing --warmup $w > $O/r${r}_w$w.json
    python3 -c "import json; b=json.load(open('$O/r${r}_w$w.json')); print('rep $r warmup $w | %.3f ms/step %.0f Mpix/s' % (b['ms_per_step'], b['value']))"
  done
done
