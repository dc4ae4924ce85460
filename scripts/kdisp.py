#!/usr/bin/env python3
"""Per-dispatch durations of the kernels whose names start with PREFIX in a rocprofv3 kernel
trace directory: every dispatch in order, then count / mean / min / max / stddev (us).
usage: python3 scripts/kdisp.py TRACE_DIR PREFIX [--json OUT]"""
import csv
import glob
import json
import statistics
import sys


def main():
    d, pre = sys.argv[1], sys.argv[2]
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not f:
        sys.exit(f"no kernel trace under {d}")
    res = {}
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        if not name.startswith(pre):
            continue
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        res.setdefault(name, []).append(round(us, 2))
    out = {}
    for k, v in res.items():
        out[k] = {"dispatches": len(v), "mean_us": round(statistics.mean(v), 2),
                  "min_us": min(v), "max_us": max(v),
                  "stddev_us": round(statistics.pstdev(v), 2), "each_us": v}
        print(k, {a: b for a, b in out[k].items() if a != "each_us"})
        print("  ", v)
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
