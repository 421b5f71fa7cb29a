"""Per-push kernel timeline from a rocprofv3 kernel trace (gpurun_out/prof/run_kernel_trace.csv): durations
and the idle gap before each launch, for the last complete push (k_stats to k_stats)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_stats<" in r["Kernel_Name"] or "k_stats(" in r["Kernel_Name"]]
seg = rows[idx[-2]:idx[-1] + 1]
t0 = int(seg[0]["Start_Timestamp"])
prev = None
busy = 0
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {gap:7.1f}  {r['Kernel_Name'].split('(')[0][-44:]}")
    prev = e
    busy += e - s
print(f"push-to-push {(int(seg[-1]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
