#!/bin/bash
# C5 through quant_rows_device with NSHARD virtual row shards, under
# rocprofv3 kernel stats, for several library builds on one box: the
# average / total time of the top kernels per build.
#   bash tools/gpu_c5_kernels.sh TAG NSHARD LIB...     (LIB: a .so path, or "tree")
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
NS=$2
shift 2
mkdir -p $O
cd $R
K='import csv,sys; rows=sorted(csv.DictReader(open(sys.argv[1])),key=lambda r:-float(r["TotalDurationNs"])); print(" | ".join("%s %s x %.1f us" % (r["Name"].split("(")[0].replace("void dq::",""), r["Calls"], float(r["AverageNs"])/1e3) for r in rows[:8]))'
for L in "$@"; do
  t=$(basename $L .so)
  if [ "$L" = tree ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/$L; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/$t -o run -- python3 -u tools/c5_shards.py $NS 3 2> $O/${t}_calls.txt > /dev/null || { tail -5 $O/${t}_calls.txt; exit 1; }
  echo "$t: $(grep -v rocprofv3 $O/${t}_calls.txt | grep call | tail -1)"
  echo "   $(python3 -c "$K" $O/$t/run_kernel_stats.csv)"
done
