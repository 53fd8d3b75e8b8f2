"""Kernel timeline of a rocprofv3 --kernel-trace CSV: the last `window` us of
kernels (or those after the first kernel matching --from), with start
offsets, durations and the idle gap before each, plus per-name totals.

    python tools/timeline.py <..._kernel_trace.csv> [--last N] [--from NAME]
"""
import argparse
import csv
import re


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = name.replace("void ", "").replace("dq::", "")
    return name[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--last", type=int, default=80, help="kernels at the end of the trace")
    ap.add_argument("--calls", type=int, default=1, help="split the tail at the map kernels")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    tail = rows[-a.last:]
    t0 = tail[0][0]
    prev_end = tail[0][0]
    busy = 0
    tot = {}
    for s, e, n in tail:
        gap = s - prev_end
        print("%9.1f  %7.1f  gap %7.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, n))
        prev_end = max(prev_end, e)
        busy += e - s
        tot[n] = tot.get(n, 0) + (e - s)
    span = tail[-1][1] - t0
    print("span %.1f us, kernel busy %.1f us (%.0f%%)" % (span / 1e3, busy / 1e3, 100.0 * busy / span))
    for n, v in sorted(tot.items(), key=lambda x: -x[1]):
        print("  %8.1f us  %s" % (v / 1e3, n))


if __name__ == "__main__":
    main()
