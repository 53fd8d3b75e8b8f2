# usage: bash tools/bh_variants.sh v1 v2 ... : bench_blockhist kernel times per library variant
set -e -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/bhv; mkdir -p $O; cd /tmp
for v in base "$@"; do
  L=$R/clusteringsegmentation-1_amd/libdivquant_hip.so
  [ "$v" != base ] && L=$R/clusteringsegmentation-1_amd/variants/$v/libdivquant_hip.so
  DQ_HIP_LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v -o p --output-format csv -- python3 $R/tools/bench_blockhist.py --cpu 0 > $O/$v.log 2>&1
  echo "== $v"; grep -h block $O/$v/p_kernel_stats.csv | cut -d, -f1-4
done
