#!/bin/bash
# Round-2 kernel work: parity, then per-kernel stats of the variants, a tile
# sweep of the passes, and PMC counters of the streaming kernels.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2a
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash tools/prof_variants.sh ${VARIANTS:-} 2>&1 | tee $O/variants.txt
for cfg in "DQ_HIP_TILES=2048" "DQ_HIP_TILES=512"; do
  env $cfg timeout -k 10 120 python bench.py --lanes 1 --no-cpu-baseline --no-c3 --no-rowtile --no-verify --steps 10 > $O/t.json
  python3 -c "
import json; d=json.load(open('$O/t.json')); k=d['detail']['kernels']
print('$cfg', d['ms_per_step'], ' '.join('%s %.1fus' % (n, v['ms']*1e3/v['launches']) for n, v in k.items() if v['launches']))" | tee -a $O/tiles.txt
done
cd $R
PMC_FULL=1 bash tools/pmc_bench.sh r2a/pmc --lanes 1 > $O/pmc.log 2>&1
python3 tools/pmc_table.py $O/pmc "partsplit|pass_kernel|map_lds" > $O/pmc_table.txt
cat $O/pmc_table.txt | head -80
