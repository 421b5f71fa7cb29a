"""Print a rocprofv3 kernel_stats.csv compactly: short kernel name, calls, total ms, average us."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 20]:
    name = r["Name"].split("(")[0].replace("void ", "")[-60:]
    print(f"{name:60s} {int(r['Calls']):7d} {int(r['TotalDurationNs']) / 1e6:9.3f} ms {float(r['AverageNs']) / 1e3:9.1f} us")
