#!/usr/bin/env python3
"""Summarise scripts/profile_f64.sh output into profiles/ (committed evidence).

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of the bench run (verbatim)
  profiles/<tag>_dec_f64_profile.json  per-kernel mean durations, HBM bytes, SQ counters
  profiles/pmc_dec_f64.json         what bench.py reports as roofline.traffic

HBM bytes: FETCH_SIZE and WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ-derived).
MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports exactly half the bytes of a
wide coalesced streaming read (16 B/lane), so it is doubled; WRITE_SIZE is exact for 16-B/lane
stores but uncalibrated for other widths, so it is reported raw and the emit kernel's known
store volume (16 B per record) is given beside it.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# a stream of frames (bench.py's timed region): one nxg_f64r_fused_kernel launch per decode (the
# emit of frame j + the probe of frame j + 1); one call per frame: probe + emit (the comparison
# leg)
FUSED = "nxg_f64r_fused_kernel"
DEC = (FUSED,)
ALL = ("nxg_f64r_probe_kernel", "nxg_f64r_emit_kernel", FUSED)


def rows(pattern):
    fs = glob.glob(pattern, recursive=True)
    return list(csv.DictReader(open(fs[0]))) if fs else []


def short(name):
    return name.split("(")[0].split("::")[-1]


def per_dispatch(rs):
    d = defaultdict(dict)
    names = {}
    for r in rs:
        k = int(r["Dispatch_Id"])
        names[k] = short(r["Kernel_Name"])
        d[k][r["Counter_Name"]] = d[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return d, names


def main():
    out, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    trace = rows(os.path.join(out, "trace", "**", "*kernel_trace.csv"))
    bench = json.load(open(os.path.join(out, "trace_bench.json")))
    records = bench["config"]["records_per_gpu"]
    dur = defaultdict(list)
    for r in trace:
        dur[short(r["Kernel_Name"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    summary = {"records": records, "wire_bytes": bench["config"]["wire_bytes_per_gpu"],
               "bench_kernel_ms": bench["roofline"]["kernel_ms"], "kernels": {}}
    for k in ALL:
        v = dur.get(k, [])
        summary["kernels"][k] = {"dispatches": len(v),
                                 "mean_us": round(sum(v) / len(v), 2) if v else None}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write"), (None, "sq")):
        d, names = per_dispatch(rows(os.path.join(out, sub, "**", "*counter_collection.csv")))
        acc = defaultdict(lambda: defaultdict(list))
        for k, cs in d.items():
            if names[k] in ALL:
                for c, v in cs.items():
                    acc[names[k]][c].append(v)
        for kn, cs in acc.items():
            for c, vs in cs.items():
                summary["kernels"][kn][c] = round(sum(vs) / len(vs), 1)
    per = summary["kernels"]
    fetch = sum(2 * 1024 * per[k].get("FETCH_SIZE", 0) for k in DEC)
    write = sum(1024 * per[k].get("WRITE_SIZE", 0) for k in DEC)
    summary["hbm_read_bytes_per_decode"] = int(fetch)
    summary["hbm_write_bytes_per_decode_raw"] = int(write)
    summary["emit_store_bytes_per_decode"] = 16 * records
    summary["decode_us_from_trace"] = round(sum(per[k]["mean_us"] or 0 for k in DEC), 2)
    json.dump(summary, open(os.path.join(prof, f"{tag}_dec_f64_profile.json"), "w"), indent=1)
    pmc = {"records": records, "kernel": FUSED,
           "hbm_bytes_per_launch": int(fetch + write),
           "read_bytes": int(fetch), "write_bytes_raw": int(write),
           "source": f"profiles/{tag}_dec_f64_profile.json (FETCH_SIZE x2 per gfx950 note)"}
    name = "pmc_dec_f64.json" if records == 10_000_000 else f"pmc_dec_f64_{records}.json"
    json.dump(pmc, open(os.path.join(prof, name), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
