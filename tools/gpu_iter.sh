#!/bin/bash
# One development iteration on the GPU box: parity tests, the default bench
# line (no CPU baseline), and rocprofv3 kernel stats of a one-lane run.
#   bash tools/gpu_iter.sh TAG [pytest -k expression]
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-iter}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
K=${2:+-k "$2"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread $K > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.json; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d['detail']['kernels']
print('value %.0f ms/step %.3f c3 %.3f ms rowtile %.0f frac %.3f (%s %.1f us) verified %s' % (
    d['value'], d['ms_per_step'], d['detail']['c3']['ms_per_frame'], d['detail']['c4_rowtile']['Mpix_per_s'],
    d['roofline']['frac'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['verified']['ok']))
print(' '.join('%s %.1fus' % (n, v['ms'] * 1e3 / v['launches']) for n, v in k.items() if v['launches']))
print('bgr24', d['detail'].get('bgr24_input'))
PY
cd /tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o lanes1 --output-format csv -- python3 $R/bench.py --lanes 1 --steps 5 --warmup 2 --no-cpu-baseline --no-c3 --no-rowtile --no-bgr > $O/prof.log 2>&1
python3 - $O/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('%-60s %5s calls avg %9.1f us  min %9.1f  max %9.1f' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3,
          float(r['MinNs']) / 1e3, float(r['MaxNs']) / 1e3))
PY
