# usage: bash tools/ab.sh REPS "ENV_A" "ENV_B" ...  -- interleaved repeats of the default bench
set -e -o pipefail
O=gpurun_out/ab; mkdir -p $O
R=$1; shift
for r in $(seq 1 $R); do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --no-timing --steps 20 --warmup 10 > $O/r${r}_$i.json
    python3 -c "import json; b=json.load(open('$O/r${r}_$i.json')); print('rep $r | $cfg | %.3f ms/step %.0f Mpix/s | c3 %.3f' % (b['ms_per_step'], b['value'], b['detail']['c3']['ms_per_frame']))"
  done
done
