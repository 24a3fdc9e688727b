"""HBM bytes per launch of one kernel from a tools/pmc.sh run, corrected as
MI355X_MICROARCH.md §HBM says:
  * FETCH_SIZE is in KiB and reads exactly half the bytes of a wide coalesced
    streaming read on gfx950 -> x 2 x 1024;
  * the counters may cover only part of the chip: SQ_WAVES counts the waves
    seen by the sampled counter instances, so the per-launch figure is scaled
    by launched_waves / SQ_WAVES.
Only dispatches of the named kernel whose FETCH_SIZE is at least 1/4 of the
largest one are averaged (the library's small self-test batch launches the
same kernels).
    python tools/make_pmc_traffic.py gpurun_out/pmc_TAG OUT.json [--kernel crc32c_fixed_kernel]
                                     [--alg-bytes B] [--blocks N] [--what TEXT]"""
import argparse, csv, glob, json, os
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("out")
ap.add_argument("--kernel", default="crc32c_fixed_kernel")
ap.add_argument("--blocks", type=int, default=100000)
ap.add_argument("--alg-bytes", type=int, default=None, help="default: blocks * (4096 + 4)")
ap.add_argument("--what", default="")
a = ap.parse_args()
vals = defaultdict(dict)  # counter -> dispatch -> value
grid = {}
for f in sorted(glob.glob(os.path.join(a.dir, "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        if a.kernel not in row["Kernel_Name"]:
            continue
        key = (f, row["Dispatch_Id"])
        vals[row["Counter_Name"]][key] = vals[row["Counter_Name"]].get(key, 0.0) + float(row["Counter_Value"])
        grid[key] = int(row["Grid_Size"])


def big(counter):
    d = vals[counter]
    top = max(d.values())
    return {k: v for k, v in d.items() if v >= top / 4}


fetch_d, write_d = big("FETCH_SIZE"), big("WRITE_SIZE")
waves = vals["SQ_WAVES"]
cov_f = sum(waves[k] / (grid[k] // 64) for k in fetch_d) / len(fetch_d)
cov_w = sum(waves[k] / (grid[k] // 64) for k in write_d) / len(write_d)
fetch = sum(fetch_d.values()) / len(fetch_d) * 1024 * 2 / cov_f
write = sum(write_d.values()) / len(write_d) * 1024 / cov_w
alg = a.alg_bytes if a.alg_bytes is not None else a.blocks * (4096 + 4)
res = {"kernel": a.kernel, "what": a.what, "blocks": a.blocks,
       "hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
       "alg_bytes_per_launch": alg, "traffic_over_alg": round((fetch + write) / alg, 4),
       "dispatches": {"fetch": len(fetch_d), "write": len(write_d)}, "coverage": round(cov_f, 4),
       "method": "FETCH_SIZE*1024*2 (gfx950 half-count on 16-B/lane streams) + WRITE_SIZE*1024, "
                 "each divided by SQ_WAVES/launched_waves (fraction of the chip the counter instances see); "
                 "separate --pmc passes, tools/pmc.sh", "source": a.dir}
json.dump(res, open(a.out, "w"), indent=1)
print(json.dumps(res, indent=1))
