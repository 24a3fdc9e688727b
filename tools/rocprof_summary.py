"""Summarise a rocprofv3 --kernel-trace run of bench.py: per-kernel-name
launch durations (all launches), and the main kernel's launches split by
bench phase in launch order -- the verification launch (1), warmup (W), timed
(K), dispatch-event pass (K), isolated pass (K), queued event-pair pass
(K) -- after dropping the
known-answer probe's small launches.
Writes the JSON summary and, with a third path, a stats CSV of the timed
phase alone (the launches bench.py's `value` and `roofline` time).

    python tools/rocprof_summary.py TRACE.csv OUT.json [STEPS WARMUP [TIMED_STATS.csv]]
"""
import csv
import json
import statistics
import sys

src, dst = sys.argv[1], sys.argv[2]
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
warm = int(sys.argv[4]) if len(sys.argv) > 4 else 5
timed_csv = sys.argv[5] if len(sys.argv) > 5 else None
rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))


def stats(d):
    return {"n": len(d), "mean_us": round(statistics.mean(d), 2), "median_us": round(statistics.median(d), 2),
            "min_us": round(min(d), 2), "max_us": round(max(d), 2)}


out = {"source": src, "steps": steps, "warmup": warm, "kernels": {}}
for name, se in by.items():
    out["kernels"][name] = stats([(e - s) / 1e3 for s, e in se])
main = max(by, key=lambda k: len(by[k]))
se = [x for x in by[main] if (x[1] - x[0]) / 1e3 > 20.0]  # drop the probe's tiny launches
d = [(e - s) / 1e3 for s, e in se]
P = 1  # bench.py's verification launch precedes the warmup
bounds = {"verify": (0, P), "warmup": (P, P + warm), "timed": (P + warm, P + warm + steps),
          "dispatch_events": (P + warm + steps, P + warm + 2 * steps),
          "isolated": (P + warm + 2 * steps, P + warm + 3 * steps),
          "queued_event_pairs": (P + warm + 3 * steps, P + warm + 4 * steps)}
out["main_kernel"] = main
out["main_phases"] = {k: stats(d[a:b]) for k, (a, b) in bounds.items() if d[a:b]}
a, b = bounds["timed"]
if len(se) >= b:
    # launch period over the timed phase, first start to last end (what the
    # bench's events bracket, minus the first launch's queueing)
    span = (se[b - 1][1] - se[a][0]) / 1e3
    out["timed_period_us"] = round(span / steps, 2)
json.dump(out, open(dst, "w"), indent=1)
if timed_csv and "timed" in out["main_phases"]:
    t = out["main_phases"]["timed"]
    dt = d[a:b]
    with open(timed_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "MedianNs"])
        w.writerow([main, t["n"], int(sum(dt) * 1e3), int(t["mean_us"] * 1e3), 100.0, int(t["min_us"] * 1e3),
                    int(t["max_us"] * 1e3), int(t["median_us"] * 1e3)])
print(json.dumps({"main_phases": out["main_phases"], "timed_period_us": out.get("timed_period_us")}))
