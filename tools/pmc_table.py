#!/usr/bin/env python3
"""Per-kernel averages of every counter in rocprofv3 --pmc CSVs under a directory.

    python tools/pmc_table.py gpurun_out/TAG [kernel-regex]

One line per (kernel, counter): average value per dispatch and the dispatch
count.  Development tool (profiles/ keeps its output as text)."""
import collections
import csv
import glob
import os
import re
import sys


def main():
    src = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for f in glob.glob(os.path.join(src, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dq::", "")
            if pat and not pat.search(name):
                continue
            key = (name, r["Counter_Name"])
            tot[key] += float(r["Counter_Value"])
            cnt[key] += 1
    last = None
    for (k, c) in sorted(tot):
        if k != last:
            print(k)
            last = k
        print("    %-28s %16.1f  (%d dispatches)" % (c, tot[(k, c)] / cnt[(k, c)], cnt[(k, c)]))


if __name__ == "__main__":
    main()
