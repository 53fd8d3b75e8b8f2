# usage: bash tools/prof_variants.sh v1 v2 ... : per-kernel averages (rocprofv3 kernel stats) of
# `bench.py --lanes 1` for the in-tree library (base) and each variants/<v>/ library
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/profv; mkdir -p $O; cd /tmp
for v in base "$@"; do
  L=$R/clusteringsegmentation-1_amd/libdivquant_hip.so
  [ "$v" != base ] && L=$R/clusteringsegmentation-1_amd/variants/$v/libdivquant_hip.so
  DQ_HIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o p --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-verify --no-timing > $O/$v.log 2>&1
  echo "== $v $(python3 -c "import json;d=json.loads(open('$O/$v.log').read().strip().splitlines()[-1]);print(d['ms_per_step'])" 2>/dev/null)"
  python3 -c "
import csv
for r in list(csv.DictReader(open('$O/$v/p_kernel_stats.csv')))[:9]:
    print('  %-60s %5s calls %9.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
done
