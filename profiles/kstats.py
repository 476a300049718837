#!/usr/bin/env python3
"""Per-kernel table of one or more rocprofv3 --kernel-trace --stats directories:
    python3 profiles/kstats.py gpurun_out/TAG/x_trace [...] [--top N]"""
import csv
import glob
import re
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 16
    for d in args:
        if d.isdigit():
            continue
        for p in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
            rows = list(csv.DictReader(open(p)))
            print("==", d)
            for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
                name = re.sub(r"\(.*", "", r["Name"]).replace("void ", "")[:44]
                print(f"  {name:44s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:9.1f} us "
                      f"total {float(r['TotalDurationNs']) / 1e6:8.2f} ms")


if __name__ == "__main__":
    main()
