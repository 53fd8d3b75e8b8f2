#!/bin/bash
# Kernel stats (rocprofv3) of the one-lane bench for library variants built by
# tools/build_variant.sh: bash tools/prof_variants.sh TAG NAME [NAME ...]
# ("default" = the in-tree library).  Prints each kernel's average per variant.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp
for v in "$@"; do
  if [ "$v" = default ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/clusteringsegmentation-1_amd/variants/$v.so; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o k --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-verify > $O/prof_$v.log 2>&1
  python3 - $O/prof_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if 'copyBuffer' not in r['Name']]
print('%-10s ' % sys.argv[2] + '  '.join('%s %.1f' % (r['Name'].split('(')[0].replace('void ', '').replace('dq::', '')[:18],
      float(r['AverageNs']) / 1e3) for r in rows[:6]))
PY
done
