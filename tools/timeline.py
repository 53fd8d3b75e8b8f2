"""Device timeline of the last N dispatches of a rocprofv3 --kernel-trace run.

    python3 tools/timeline.py PROF_DIR [N]

One line per dispatch: start (us, from the first shown), duration, gap to the
previous dispatch's end, kernel; then the span, the busy time and the time
per kernel name."""
import collections
import csv
import glob
import os
import sys


def main():
    path = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)
    if not path:
        raise SystemExit("no kernel_trace.csv under %s" % sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    rows = list(csv.DictReader(open(path[0])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)[-n:]
    t0 = ev[0][0]
    prev_end = None
    busy = 0.0
    per = collections.Counter()
    for s, e, name in ev:
        short = name.replace("dq::", "").split("(")[0].replace("void ", "")
        gap = 0.0 if prev_end is None else (s - prev_end) / 1e3
        print("%9.1f %8.1f  gap %6.1f  %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, short))
        prev_end = e if prev_end is None else max(prev_end, e)
        busy += (e - s) / 1e3
        per[short] += (e - s) / 1e3
    span = (ev[-1][1] - t0) / 1e3
    print("span %.1f us, kernel busy %.1f us (%d%%)" % (span, busy, round(100 * busy / span)))
    for k, v in per.most_common():
        print("%10.1f us  %s" % (v, k))


if __name__ == "__main__":
    main()
