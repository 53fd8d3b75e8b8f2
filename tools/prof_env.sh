# usage: bash tools/prof_env.sh "ENV=.." ... : partsplit / total kernel averages per env setting
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/profe; mkdir -p $O; cd /tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/e$i -o p --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-timing > $O/e$i.log 2>&1
  python3 -c "
import csv
rows=list(csv.DictReader(open('$O/e$i/p_kernel_stats.csv')))
tot=sum(float(r['TotalDurationNs']) for r in rows)/7/1e3
ps=[r for r in rows if 'partsplit' in r['Name']][0]
print('$cfg | partsplit %.1f us x %s | kernels per call %.0f us' % (float(ps['AverageNs'])/1e3, ps['Calls'], tot))"
done
