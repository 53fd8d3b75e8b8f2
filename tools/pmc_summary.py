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
RANGE = {}   # counter -> kernel -> (min, max) per dispatch, KiB


def per_kernel(path, counter, by_grid=None):
    """{kernel: (mean value, dispatches)}; by_grid (a dict) also gets
    {kernel: {grid size: (mean, dispatches)}} -- one 4K frame's map and an
    8-frame batch's map are different dispatches of one kernel, and so are
    the partition's modes, so an average over all of them is no byte count of
    any one (evidence hygiene)."""
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    gtot = collections.defaultdict(float)
    gcnt = collections.defaultdict(int)
    vmin, vmax = {}, {}
    for f in glob.glob(os.path.join(path, "**", "*_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dq::", "")
            name = name.replace("<0>", "<PASS_INIT>").replace("<1>", "<PASS_SPLIT>")
            name = name.replace("<2>", "<PASS_KMEANS>").replace("<3>", "<PASS_KLAST>")
            name = name.replace("<false>", "").replace("<true>", "")
            v = float(r["Counter_Value"])
            tot[name] += v
            cnt[name] += 1
            vmin[name] = min(vmin.get(name, v), v)
            vmax[name] = max(vmax.get(name, v), v)
            gk = (name, int(r["Grid_Size"]))
            gtot[gk] += float(r["Counter_Value"])
            gcnt[gk] += 1
    out = {k: (tot[k] / cnt[k], cnt[k]) for k in tot}
    for k in tot:   # the spread of the per-dispatch values (a mixed average shows as a wide one)
        RANGE.setdefault(counter, {})[k] = (vmin[k], vmax[k])
    if by_grid is not None:
        for (name, grid), t in gtot.items():
            by_grid.setdefault(name, {})[grid] = (t / gcnt[(name, grid)], gcnt[(name, grid)])
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
    fg, wg = {}, {}
    fetch = per_kernel(src, "FETCH_SIZE", fg)
    write = per_kernel(src, "WRITE_SIZE", wg)
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(out_path)) if os.path.exists(out_path) else {}
    entry = {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, (0.0, 0))[0] * 1024 * 2
        wb = write.get(k, (0.0, 0))[0] * 1024
        entry[k] = {"hbm_bytes_per_launch": fb + wb, "read_bytes_per_launch": fb,
                    "write_bytes_per_launch": wb, "dispatches": fetch.get(k, (0, 0))[1],
                    "source": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + WRITE_SIZE: %s" % src.rstrip("/")}
        if k in RANGE.get("FETCH_SIZE", {}):
            lo, hi = RANGE["FETCH_SIZE"][k]
            entry[k]["read_bytes_per_dispatch_min_max"] = [lo * 1024 * 2, hi * 1024 * 2]
        if k in RANGE.get("WRITE_SIZE", {}):
            lo, hi = RANGE["WRITE_SIZE"][k]
            entry[k]["write_bytes_per_dispatch_min_max"] = [lo * 1024, hi * 1024]
        if k in fg:   # per dispatch size (grid = workgroups x threads)
            entry[k]["by_grid_size"] = {
                str(g): {"hbm_bytes_per_launch": fv * 1024 * 2 + wg.get(k, {}).get(g, (0.0, 0))[0] * 1024,
                         "read_bytes_per_launch": fv * 1024 * 2,
                         "write_bytes_per_launch": wg.get(k, {}).get(g, (0.0, 0))[0] * 1024,
                         "dispatches": c}
                for g, (fv, c) in sorted(fg[k].items())}
    db[key] = entry
    json.dump(db, open(out_path, "w"), indent=1, sort_keys=True)
    for k, v in entry.items():
        print("%-28s %14.0f B/launch (read %.0f, write %.0f) over %d dispatches"
              % (k, v["hbm_bytes_per_launch"], v["read_bytes_per_launch"], v["write_bytes_per_launch"], v["dispatches"]))


if __name__ == "__main__":
    main()
