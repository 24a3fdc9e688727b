"""Last kernels of a rocprofv3 kernel trace as a timeline (start offset and
duration, us).  python tools/diag/ktl.py gpurun_out/tdt/run_kernel_trace.csv [N]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-int(sys.argv[2] if len(sys.argv) > 2 else 14):]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {r['Kernel_Name'][:80]}")
