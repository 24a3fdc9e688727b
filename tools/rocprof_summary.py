"""Summarise a rocprofv3 --kernel-trace run of bench.py: per-kernel-name
launch durations (all launches, and the main-kernel launches split by bench
phase: warmup / timed / bracketed), written next to the stats CSV.
    python tools/rocprof_summary.py gpurun_out/prof_TAG/run_kernel_trace.csv out.json [steps warmup]"""
import csv, json, statistics, sys
src, dst = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 5
rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {"source": src, "kernels": {}}
for name, d in by.items():
    out["kernels"][name] = {"calls": len(d), "mean_us": round(statistics.mean(d), 2),
                            "median_us": round(statistics.median(d), 2), "min_us": round(min(d), 2),
                            "max_us": round(max(d), 2)}
main = max(by, key=lambda k: len(by[k]))
d = [x for x in by[main] if x > 20.0]  # drop the self-test's tiny launches
ph = {"warmup": d[:warm], "timed": d[warm:warm + steps], "bracketed": d[warm + steps:]}
out["main_kernel"] = main
out["main_phases"] = {k: {"n": len(v), "mean_us": round(statistics.mean(v), 2), "median_us": round(statistics.median(v), 2)}
                      for k, v in ph.items() if v}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["main_phases"]))
