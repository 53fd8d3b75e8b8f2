#!/bin/bash
# Quick GPU check: parity tests, the bench line, per-kernel stats of variants.
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-quick}; shift || true
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-rowtile > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; cat $O/bench.json; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); k=d['detail']['kernels']
print('value', d['value'], 'ms/step', d['ms_per_step'], 'c3', d['detail']['c3']['ms_per_frame'], 'frac', d['roofline']['frac'], d['roofline']['kernel'])
print(' '.join('%s %.1fus' % (n, v['ms']*1e3/v['launches']) for n, v in k.items() if v['launches']))"
bash tools/prof_variants.sh "$@" 2>&1 | tee $O/variants.txt
