#!/bin/bash
# GPU suite, then map_colors_mps alone (tools/mapbench.py) under kernel
# stats for library variants and DQ_HIP_TUNE settings.
#   bash tools/gpu_map_ab.sh TAG "VAR VAR.." "TUNE TUNE.."
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
run() {   # NAME: one mapbench under rocprofv3 kernel stats
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/$1 -o run -- python3 -u tools/mapbench.py 20 > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  echo "$1 $(cat $O/$1.json) $(grep 'map_lds\|build_cells' $O/$1/run_kernel_stats.csv | cut -d, -f1-4 | tr '\n' ' ')"
}
for v in $2; do
  if [ "$v" = tree ]; then unset DQ_HIP_LIB; else export DQ_HIP_LIB=$R/tools/bin/$v.so; fi
  run $v
done
unset DQ_HIP_LIB
for t in $3; do
  DQ_HIP_TUNE=$t run tune_$t
done
echo map ab done
