#!/bin/bash
# The hand-off experiment of DESIGN.md 3b: the C4 share under prewarm (+ uneven)
# with the round-3 protocol (the library) and with round 2's (a build of the
# round-2 kpass hand-off, variants/libdq_r2proto.so), 10 calls each.
set -e -o pipefail
O=$1
timeout -k 10 240 python -u tools/handoff_experiment.py 3 10 > $O/exp_new.jsonl 2>&1 || { tail $O/exp_new.jsonl; exit 1; }
tail -1 $O/exp_new.jsonl
DQ_HIP_LIB=clusteringsegmentation-1_amd/variants/libdq_r2proto.so timeout -k 10 240 \
  python -u tools/handoff_experiment.py 3 10 > $O/exp_r2.jsonl 2>&1 || { tail $O/exp_r2.jsonl; exit 1; }
tail -1 $O/exp_r2.jsonl
