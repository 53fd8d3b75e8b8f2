#!/usr/bin/env bash
# Builds oracle/_ref/libdqref_instr.so: a SCRATCH copy of the reference DivQuant
# sources (copied to a temp dir that is deleted afterwards, never committed)
# with two fprintf(stderr) lines inserted, as SURVEY 8c prescribes:
#   DQTRACE new_index old_index |C| |new|   after DivQuantCluster.cpp:821
#   DQMEAN  ic mean.r mean.g mean.b (%a)    inside the size>0 block, :1053
# Used only by tests/golden/make_golden.py to pin split traces and the double
# centroids (the north star's 1e-5 check) to the reference itself.
set -euo pipefail
REF=${REF:-/root/reference/DivQuant}
HERE=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d)
trap 'rm -rf "$TMP"' EXIT
cp "$REF"/*.cpp "$REF"/*.h "$TMP"/
f="$TMP/DivQuantCluster.cpp"
grep -q '    size\[new_index\] = new_size;' "$f"
grep -q '      uint32_t pixel = (R << 16) | (G << 8) | B;' "$f"
sed -i 's|^    size\[new_index\] = new_size;$|    size[new_index] = new_size; fprintf(stderr, "DQTRACE %d %d %d %d\\n", new_index, old_index, tmp_num_points, new_size);|' "$f"
sed -i 's|^      uint32_t pixel = (R << 16) \| (G << 8) \| B;$|      uint32_t pixel = (R << 16) \| (G << 8) \| B; fprintf(stderr, "DQMEAN %d %a %a %a\\n", ic, mean[ic].red, mean[ic].green, mean[ic].blue);|' "$f"
[ "$(grep -c DQTRACE "$f")" = 1 ] && [ "$(grep -c DQMEAN "$f")" = 1 ]
mkdir -p "$HERE/oracle/_ref"
g++ -O2 -std=c++11 -fPIC -shared -include stdint.h -include algorithm -I"$TMP" \
    -o "$HERE/oracle/_ref/libdqref_instr.so" "$TMP"/DivQuantCluster.cpp "$TMP"/DivQuantMapColors.cpp \
    "$TMP"/DivQuantMisc.cpp "$TMP"/DivQuantUni.cpp "$TMP"/quant_util.cpp -lz
echo "built $HERE/oracle/_ref/libdqref_instr.so"
