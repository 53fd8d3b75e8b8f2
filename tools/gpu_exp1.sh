#!/bin/bash
# Round 6 experiment: partition / copy rates at frame-sized (Infinity-Cache
# resident) inputs, and the 8 x 4K share with each lane's frames run one at
# a time (DQ_HIP_TUNE lane_frames=1) against the default.  (lane_frames was a
# key of the experiment build only, removed after it measured 1.41 vs 1.13 ms.)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/exp1
mkdir -p $O
cd $R
L=$R/clusteringsegmentation-1_amd/libdivquant_hip.so
for N in 8294400 16588800 33177600 66355200; do
  echo "== N $N" | tee -a $O/ps.txt
  timeout -k 10 120 tools/bin/psbench $L $N 20 8,64 full,stats 16 2>&1 | tee -a $O/ps.txt
done
B="python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-timing --no-c3 --no-weighted --no-c2 --no-c5 --no-rowtile --no-bgr"
for t in "" "lane_frames=1" "" "lane_frames=1"; do
  echo "== tune '$t'" | tee -a $O/bench.txt
  DQ_HIP_TUNE="$t" timeout -k 10 240 $B 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['verified'])" | tee -a $O/bench.txt
done
echo done
