#!/bin/bash
# Build tools/bin/psb_<name> variants of the partsplit microbench:
#   bash tools/build_psb.sh name "-DFLAG=1 ..." [name2 "flags2" ...]
set -e
cd "$(dirname "$0")/.."
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off $2 -o tools/bin/psb_$1 tools/psbench.hip 2>&1 | grep -v hip-link || true
  shift 2
done
ls tools/bin
