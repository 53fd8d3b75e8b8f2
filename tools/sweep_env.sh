# usage: bash tools/sweep_env.sh "ENV=.." "ENV=.." ...   (bench --lanes 1 and default lanes per setting)
set -e -o pipefail
O=gpurun_out/envs; mkdir -p $O
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python bench.py --lanes 1 --no-cpu-baseline --no-c3 --steps 10 > $O/l1_$i.json
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline --steps 10 > $O/l3_$i.json
  python3 -c "
import json; a=json.load(open('$O/l1_$i.json')); b=json.load(open('$O/l3_$i.json')); k=a['detail']['kernels']
print('$cfg | lanes1 %.3f ms | lanes3 %.3f ms (%.0f Mpix/s) | c3 %s | km %.0f us/step epi %.0f part %.0f' % (a['ms_per_step'], b['ms_per_step'], b['value'], b['detail']['c3']['ms_per_frame'], k['pass_kmeans']['ms']*100, k['epilogue']['ms']*100, k['partition']['ms']*100))"
done
