#!/bin/bash
# Run every tools/bin/psb_* variant: planar cut, planar plane, packed cut.
# (a failed check -- rc 1, expected for ablations -- is reported, not fatal)
set -o pipefail
cd "$(dirname "$0")/.."
for b in tools/bin/psb_*; do
  echo "== $(basename $b)"
  for args in ${PSB_ARGS:-"66355200,1,1" "66355200,1,0" "66355200,0,1"}; do
    timeout -k 5 60 $b ${args//,/ }
    rc=$?
    if [ $rc -gt 1 ]; then echo "CRASH rc=$rc"; exit 1; fi
  done
done
