"""Where a routed call's time goes: from a rocprofv3 --kernel-trace CSV, every
crc32c_route_plan -> crc32c_route_kernel -> crc32c_var_fused_kernel triple
(in launch order), median durations of the three kernels, the gaps between
them, and plan start -> fused end; the single region kernel's median beside.
    python tools/diag/route_tl.py TRACE.csv
"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
trip, solo = [], []
for k, (name, s, e) in enumerate(ev):
    if "crc32c_region_kernel" in name:
        solo.append((e - s) / 1e3)
    if "crc32c_route_plan" in name and k + 2 < len(ev) and "crc32c_route_kernel" in ev[k + 1][0] \
            and "crc32c_var_fused_kernel" in ev[k + 2][0]:
        (_, s1, e1), (_, s2, e2) = ev[k + 1], ev[k + 2]
        trip.append(((e - s) / 1e3, (s1 - e) / 1e3, (e1 - s1) / 1e3, (s2 - e1) / 1e3, (e2 - s2) / 1e3, (e2 - s) / 1e3))
med = lambda xs: round(statistics.median(xs), 2) if xs else None
if trip:
    cols = list(zip(*trip))
    print({"routed_calls": len(trip), "plan_us": med(cols[0]), "gap_plan_route_us": med(cols[1]),
           "route_kernel_us": med(cols[2]), "gap_route_fused_us": med(cols[3]), "fused_us": med(cols[4]),
           "total_us": med(cols[5])})
print({"region_kernel_launches": len(solo), "region_kernel_us": med(solo)})
