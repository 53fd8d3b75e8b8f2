#!/bin/bash
# Library variants for tools/psbench (development tool): dq_kernels.hip with
# extra -D flags, linked with the tree's other objects.
#   bash tools/psvar.sh NAME "-DFLAG=V ..."   -> tools/bin/NAME.so
set -e
R=$(cd $(dirname $0)/.. && pwd)
B=$R/clusteringsegmentation-1_amd/build
mkdir -p $R/tools/bin/obj
make -s -C $R/clusteringsegmentation-1_amd >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function $2 \
  -c -o $R/tools/bin/obj/$1.o $R/clusteringsegmentation-1_amd/csrc/dq_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/tools/bin/$1.so $R/tools/bin/obj/$1.o $B/dq_weighted.o $B/dq_engine.o \
  $B/dq_abi.o $B/build_id.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built tools/bin/$1.so
