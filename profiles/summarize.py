#!/usr/bin/env python3
"""Summarise one profiles/collect.sh run (gpurun_out/<tag>/) into profiles/<tag>_*.

    python profiles/summarize.py r01c [--src gpurun_out]

Writes
  <tag>_kernel_stats.csv   the rocprofv3 --kernel-trace --stats table, as collected
  <tag>_kernel_stats.md    per kernel: calls, average duration, share, and the PMC passes
                           (FETCH_SIZE x2, WRITE_SIZE, SQ issue counters) averaged per launch
  <tag>_pmc.json           k_find_sorted's HBM bytes per launch and its issue rates (bench.py reads
                           the newest one whose "config" matches its workload for the roofline)
  <tag>_bench.json         the bench.py JSON line of the same run

FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: gfx950 tallies 128-B requests at 64 B);
WRITE_SIZE is taken as reported.  Both are kilobytes per dispatch in rocprofv3's CSV.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import re
import shutil
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name)
    return name.replace("void ", "").strip()


def pmc(path: str):
    """kernel -> counter -> (sum, launches); the pseudo-counter "_ns" sums each dispatch's duration"""
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, set()]))
    if not os.path.exists(path):
        return acc
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short(row["Kernel_Name"])
            if not k.startswith("sz4::"):
                continue
            a = acc[k][row["Counter_Name"]]
            a[0] += float(row["Counter_Value"])
            a[1].add(row["Dispatch_Id"])
            d = acc[k]["_ns"]
            if row["Dispatch_Id"] not in d[1] and row.get("End_Timestamp"):
                d[0] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                d[1].add(row["Dispatch_Id"])
    return acc


def per_launch(acc, k, c):
    v = acc.get(k, {}).get(c)
    if not v or not v[1]:
        return None
    return v[0] / len(v[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--workload", default="enwik8")
    ap.add_argument("--bytes-per-gpu", type=int, default=100_000_000)
    ap.add_argument("--block-size", type=int, default=65536)
    a = ap.parse_args()
    src = os.path.join(a.src, a.tag)
    stats = os.path.join(src, "trace", "bench_kernel_stats.csv")
    rows = []
    with open(stats) as f:
        for r in csv.DictReader(f):
            if short(r["Name"]).startswith("sz4::"):
                rows.append(r)
    shutil.copy(stats, os.path.join(HERE, f"{a.tag}_kernel_stats.csv"))
    fetch = pmc(os.path.join(src, "fetch", "bench_counter_collection.csv"))
    write = pmc(os.path.join(src, "write", "bench_counter_collection.csv"))
    sq = pmc(os.path.join(src, "sq", "bench_counter_collection.csv"))

    def fmt(v, scale=1.0, p=1):
        return "-" if v is None else (f"{v * scale:.{p}f}" if scale != "e" else f"{v:.3g}")

    lines = [f"# {a.tag} kernel profile (bench.py workload {a.workload}: {a.bytes_per_gpu / 1e6:g} MB, "
             f"{a.block_size // 1024} KiB blocks, -9)", "",
             f"Source: `bash profiles/collect.sh {a.tag}` on one MI355X, summarised by "
             f"`python profiles/summarize.py {a.tag}` (rocprofv3 --kernel-trace --stats; every PMC pass separate).",
             "FETCH_SIZE doubled per MI355X_MICROARCH.md; MB = 1e6 bytes per launch.", "",
             "| kernel | calls | avg us | % | FETCH x2 (MB) | WRITE (MB) | VALU instr | SALU instr | LDS instr | wait-any % |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    find = None
    for r in rows:
        k = short(r["Name"])
        fe = per_launch(fetch, k, "FETCH_SIZE")
        wr = per_launch(write, k, "WRITE_SIZE")
        valu = per_launch(sq, k, "SQ_INSTS_VALU")
        salu = per_launch(sq, k, "SQ_INSTS_SALU")
        lds = per_launch(sq, k, "SQ_INSTS_LDS")
        wc = per_launch(sq, k, "SQ_WAVE_CYCLES")
        wa = per_launch(sq, k, "SQ_WAIT_ANY")
        wait = None if not wc or wa is None else 100.0 * wa / wc
        lines.append(f"| {k} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.1f} | "
                     f"{fmt(fe, 2 * 1024 / 1e6)} | {fmt(wr, 1024 / 1e6)} | {fmt(valu, 'e')} | {fmt(salu, 'e')} | "
                     f"{fmt(lds, 'e')} | {fmt(wait, 1.0, 0)} |")
        if k.startswith("sz4::k_find_sorted"):
            find = (k, float(r["AverageNs"]), fe, wr, valu, salu)
    with open(os.path.join(HERE, f"{a.tag}_kernel_stats.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    bench = os.path.join(src, "bench.json")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(HERE, f"{a.tag}_bench.json"))
    if find:
        k, avg_ns, fe, wr, valu, salu = find
        fb = None if fe is None else int(round(fe * 1024 * 2))
        wb = None if wr is None else int(round(wr * 1024))
        cycles = avg_ns * 1e-9 * 2.4e9  # MI355X_MICROARCH.md: 2.4 GHz
        # the clock the kernel actually ran at, from the SQ pass itself: GRBM_GUI_ACTIVE is summed over the
        # 8 XCDs (MI355X_MICROARCH.md, DVFS give-back), so cycles per launch = GRBM_GUI_ACTIVE / 8, and the
        # same pass's dispatch durations give the clock
        grbm = per_launch(sq, k, "GRBM_GUI_ACTIVE")
        sq_ns = per_launch(sq, k, "_ns")
        sq_cycles = None if grbm is None else grbm / 8.0
        clock = None if sq_cycles is None or not sq_ns else sq_cycles / sq_ns
        out = {"kernel": "k_find_sorted", "tag": a.tag,
               "config": {"workload": a.workload, "bytes_per_gpu": a.bytes_per_gpu, "block_size": a.block_size,
                          "level": 9},
               "avg_duration_us": round(avg_ns / 1e3, 1),
               "fetch_bytes_corrected": fb, "write_bytes": wb,
               "hbm_bytes_per_launch": None if fb is None or wb is None else fb + wb,
               "valu_per_simd_cycle": None if valu is None else round(valu / (cycles * 1024), 4),
               "salu_per_cu_cycle": None if salu is None else round(salu / (cycles * 256), 4),
               "clock_ghz_measured": None if clock is None else round(clock, 3),
               "valu_per_simd_cycle_at_clock": None if valu is None or not sq_cycles else round(valu / (sq_cycles * 1024), 4),
               "salu_per_cu_cycle_at_clock": None if salu is None or not sq_cycles else round(salu / (sq_cycles * 256), 4),
               "method": "rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE and an SQ pass, each a separate run "
                         "(profiles/collect.sh); FETCH_SIZE doubled per MI355X_MICROARCH.md; WRITE_SIZE as reported; "
                         "issue rates = SQ_INSTS_VALU / (duration x 2.4 GHz x 1024 SIMDs), "
                         "SQ_INSTS_SALU / (duration x 2.4 GHz x 256 CUs); the _at_clock rates use the SQ pass's own cycles, "
                         "GRBM_GUI_ACTIVE / 8 per launch (clock_ghz_measured = those cycles / that pass's dispatch time)"}
        with open(os.path.join(HERE, f"{a.tag}_pmc.json"), "w") as f:
            json.dump(out, f, indent=1)
            f.write("\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
