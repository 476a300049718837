#!/usr/bin/env python3
"""Summarises profiles/phase_pmc.sh: per variant and kernel, the average duration (kernel trace) and
per-launch FETCH_SIZE (doubled: MI355X_MICROARCH.md, gfx950 tallies 128-B requests at 64 B), WRITE_SIZE
and the L2 hit rate.
    python3 profiles/phase_summary.py gpurun_out/TAG [kernel-substring ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    return re.sub(r"\(.*$", "", name).replace("void ", "").strip()


def counters(d):
    acc = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                n[k].add(row["Dispatch_Id"])
    return {k: {c: v / len(n[k]) for c, v in cs.items()} for k, cs in acc.items()}


def trace(d):
    out = {}
    for path in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                out[short(row["Name"])] = (int(row["Calls"]), float(row["AverageNs"]) / 1e3)
    return out


def main():
    top = sys.argv[1]
    keys = sys.argv[2:] or ["find_sorted", "find_big", "find_long9", "dp_spec", "dp_fix"]
    variants = sorted({os.path.basename(p).rsplit("_", 1)[0] for p in glob.glob(os.path.join(top, "*_trace"))})
    for v in variants:
        tr = trace(os.path.join(top, f"{v}_trace"))
        fe = counters(os.path.join(top, f"{v}_fetch"))
        wr = counters(os.path.join(top, f"{v}_write"))
        tc = counters(os.path.join(top, f"{v}_tcc"))
        print(f"== {v}")
        for k in sorted(tr, key=lambda x: -tr[x][0] * tr[x][1]):
            if not any(s in k for s in keys):
                continue
            calls, us = tr[k]
            f = fe.get(k, {}).get("FETCH_SIZE")
            w = wr.get(k, {}).get("WRITE_SIZE")
            h, m = tc.get(k, {}).get("TCC_HIT_sum"), tc.get(k, {}).get("TCC_MISS_sum")
            fs = f"{2 * f / 1e6:.3f} GB" if f is not None else "-"
            ws = f"{w / 1e6:.3f} GB" if w is not None else "-"
            hs = f"{h / (h + m):.3f} ({(h + m) / 1e6:.1f} M req)" if h is not None and m is not None and h + m else "-"
            print(f"  {k:40s} calls {calls:4d} avg {us:10.1f} us  fetch {fs:>11s}  write {ws:>11s}  L2 hit {hs}")


if __name__ == "__main__":
    main()
