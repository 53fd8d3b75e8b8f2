#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_bench.sh)
into profiles/pmc_traffic.json: HBM bytes per launch of every kernel.

    python tools/pmc_summary.py gpurun_out/TAG KEY

KEY names the bench command the counters came from (bench.py looks up
"<mode>_<config>_f<frames>_n<gpus>").  Corrections per MI355X_MICROARCH.md
(HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a 16-B-per-lane coalesced streaming read
(global_load_dwordx4 -- every streaming kernel here), so it is doubled;
WRITE_SIZE is taken as is.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for f in glob.glob(os.path.join(path, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dq::", "")
            name = name.replace("<0>", "<PASS_INIT>").replace("<1>", "<PASS_SPLIT>")
            name = name.replace("<2>", "<PASS_KMEANS>").replace("<3>", "<PASS_KLAST>")
            name = name.replace("<false>", "").replace("<true>", "")
            tot[name] += float(r["Counter_Value"])
            cnt[name] += 1
    out = {k: (tot[k] / cnt[k], cnt[k]) for k in tot}
    # kernels specialised per (mode, format) (partsplit_kernel<0, 2>, ...): also
    # the average over all their launches under the bare name, as bench.py's
    # HIP events time them (one kind)
    base = collections.defaultdict(lambda: [0.0, 0])
    for k in tot:
        if "<" in k and "," in k:
            b = base[k.split("<")[0]]
            b[0] += tot[k]
            b[1] += cnt[k]
    for k, (t, c) in base.items():
        out.setdefault(k, (t / c, c))
    return out


def main():
    src, key = sys.argv[1], sys.argv[2]
    fetch = per_kernel(src, "FETCH_SIZE")
    write = per_kernel(src, "WRITE_SIZE")
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(out_path)) if os.path.exists(out_path) else {}
    entry = {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, (0.0, 0))[0] * 1024 * 2
        wb = write.get(k, (0.0, 0))[0] * 1024
        entry[k] = {"hbm_bytes_per_launch": fb + wb, "read_bytes_per_launch": fb,
                    "write_bytes_per_launch": wb, "dispatches": fetch.get(k, (0, 0))[1],
                    "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE: %s" % src.rstrip("/")}
    db[key] = entry
    json.dump(db, open(out_path, "w"), indent=1, sort_keys=True)
    for k, v in entry.items():
        print("%-28s %14.0f B/launch (read %.0f, write %.0f) over %d dispatches"
              % (k, v["hbm_bytes_per_launch"], v["read_bytes_per_launch"], v["write_bytes_per_launch"], v["dispatches"]))


if __name__ == "__main__":
    main()
