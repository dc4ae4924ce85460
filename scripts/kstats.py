"""Print the nxg kernels of a rocprofv3 kernel_stats.csv: calls, average / min / max microseconds."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0]
    if n.startswith("nxg") or "scan" in n:
        print(f"{n[:48]:48s} {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:9.2f} us "
              f"min {float(r['MinNs'])/1e3:9.2f} max {float(r['MaxNs'])/1e3:9.2f}")
