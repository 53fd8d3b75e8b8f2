#!/bin/bash
# Build a variant of the library with extra -D flags into
# clusteringsegmentation-1_amd/variants/NAME.so (git-ignored; travels to the
# GPU box).  Select it with DQ_HIP_LIB=<path>.
#   bash tools/build_variant.sh NAME "-DDQ_PS_PREFETCH=0 ..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/clusteringsegmentation-1_amd
mkdir -p $P/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function $2 \
  -shared -o $P/variants/$1.so $P/csrc/dq_kernels.hip $P/csrc/dq_weighted.hip $P/csrc/dq_engine.cpp $P/csrc/dq_abi.cpp \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib 2>&1 | grep -v hip-link || true
ls -la $P/variants/$1.so
