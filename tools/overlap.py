"""Stream overlap in a rocprofv3 --kernel-trace CSV: over the last `--span`
microseconds, the busy time of each stream, of their union, and the time
both streams run kernels at once; plus a compact two-column timeline of the
last `--show` kernels.  Development tool.

    python tools/overlap.py <..._kernel_trace.csv> [--span US] [--show N]
"""
import argparse
import csv
import re


def short(name):
    name = re.sub(r"\(.*$", "", name)
    return name.replace("void ", "").replace("dq::", "")[:28]


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--span", type=float, default=3000.0)
    ap.add_argument("--show", type=int, default=60)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.csv)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id") or r["Queue_Id"],
                     short(r["Kernel_Name"])))
    rows.sort()
    t_end = max(e for _, e, _, _ in rows)
    t0 = t_end - a.span * 1e3
    win = [(max(s, t0), e, q, n) for s, e, q, n in rows if e > t0]
    streams = sorted(set(q for _, _, q, _ in win))
    per = {q: union_len([(s, e) for s, e, qq, _ in win if qq == q]) for q in streams}
    uni = union_len([(s, e) for s, e, _, _ in win])
    both = sum(per.values()) - uni
    print("window %.0f us; union busy %.1f us (%.0f%%)" % (a.span, uni / 1e3, 100.0 * uni / (a.span * 1e3)))
    for q in streams:
        print("  stream %s busy %.1f us" % (q, per[q] / 1e3))
    print("  concurrent (>= 2 streams) %.1f us" % (both / 1e3))
    col = {q: i for i, q in enumerate(streams)}
    for s, e, q, n in win[-a.show:]:
        pad = " " * 44 * col[q]
        print("%9.1f %s%-28s %6.1f" % ((s - t0) / 1e3, pad, n, (e - s) / 1e3))


if __name__ == "__main__":
    main()
