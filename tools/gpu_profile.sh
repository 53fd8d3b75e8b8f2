#!/bin/bash
# Profiles of the bench's C4-share leg (8 x 4K, one engine lane: launches
# un-overlapped) from the SAME tree, in three separate runs:
#   1. rocprofv3 --kernel-trace --stats: per-kernel stats + per-launch trace,
#      with the bench line whose roofline they must agree with;
#   2. --pmc FETCH_SIZE (its own pass: it takes 3 of the 4 TCC counters);
#   3. --pmc WRITE_SIZE.
#   bash tools/gpu_profile.sh TAG      (outputs under gpurun_out/TAG)
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
B="bench.py --lanes 1 --no-c3 --no-c2 --no-c5 --no-rowtile --no-bgr --no-weighted --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $O/prof -o run -- \
  python3 -u $B > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
python3 tools/roofline_check.py $O/bench_prof.json $O/prof > $O/roofline_check.txt
cat $O/roofline_check.txt
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/pmc_fetch -o run -- \
  python3 -u $B --no-timing --steps 2 --warmup 1 > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/pmc_write -o run -- \
  python3 -u $B --no-timing --steps 2 --warmup 1 > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
echo profile done
