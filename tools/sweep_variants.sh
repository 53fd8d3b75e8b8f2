# usage: bash tools/sweep_variants.sh v1 v2 ... (dirs under clusteringsegmentation-1_amd/variants)
set -e -o pipefail
O=gpurun_out/variants; mkdir -p $O
for v in "$@"; do
  DQ_HIP_LIB=$PWD/clusteringsegmentation-1_amd/variants/$v/libdivquant_hip.so timeout -k 10 120 python bench.py --lanes 1 --no-cpu-baseline --no-c3 --steps 10 > $O/$v.json
  python3 -c "
import json; d=json.load(open('$O/$v.json')); k=d['detail']['kernels']
print('$v', d['value'], d['ms_per_step'], 'partsplit us %.1f'%(k['partition']['ms']*1e3/k['partition']['launches']), 'kmeans us %.1f'%(k['pass_kmeans']['ms']*1e3/k['pass_kmeans']['launches']), 'map us %.1f'%(k['map']['ms']*1e3/k['map']['launches']))"
done
