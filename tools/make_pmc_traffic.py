"""Derive profiles/pmc_traffic.json (HBM bytes per launch of the fast-path
kernel) from a tools/pmc.sh run, corrected as MI355X_MICROARCH.md §HBM says:
  * FETCH_SIZE is in KiB and reads exactly half the bytes of a wide coalesced
    streaming read on gfx950 -> x 2 x 1024;
  * the counters of this pool cover only part of the chip: SQ_WAVES counts the
    waves seen by the sampled counter instances (3416 of 4096 launched), so the
    per-launch figure is scaled by launched_waves / SQ_WAVES.
    python tools/make_pmc_traffic.py gpurun_out/pmc_TAG profiles/pmc_traffic.json"""
import csv, glob, json, os, sys
from collections import defaultdict
d, outp = sys.argv[1], sys.argv[2]
blocks = int(sys.argv[3]) if len(sys.argv) > 3 else 100000
vals = defaultdict(lambda: defaultdict(float))
meta = {}
for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        if "crc32c_fixed_kernel" not in row["Kernel_Name"] or int(row["Grid_Size"]) < 100000:
            continue
        vals[row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
        meta["grid_threads"] = int(row["Grid_Size"])
mean = {k: sum(v.values()) / len(v) for k, v in vals.items()}
launched_waves = meta["grid_threads"] // 64
cover = mean["SQ_WAVES"] / launched_waves
fetch = mean["FETCH_SIZE"] * 1024 * 2 / cover
write = mean.get("WRITE_SIZE", 0.0) * 1024 / cover
alg = blocks * (4096 + 4)
res = {"kernel": "crc32c_fixed_kernel<0>", "blocks": blocks, "block_bytes": 4096,
       "hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
       "alg_bytes_per_launch": alg, "traffic_over_alg": round((fetch + write) / alg, 4),
       "raw": {"FETCH_SIZE_KiB": mean["FETCH_SIZE"], "WRITE_SIZE_KiB": mean.get("WRITE_SIZE"),
               "SQ_WAVES": mean["SQ_WAVES"], "launched_waves": launched_waves, "coverage": round(cover, 4)},
       "method": "FETCH_SIZE*1024*2 (gfx950 half-count on 16-B/lane streams) + WRITE_SIZE*1024, "
                 "each divided by SQ_WAVES/launched_waves (fraction of the chip the counter instances see); "
                 "separate --pmc passes, tools/pmc.sh", "source": d}
json.dump(res, open(outp, "w"), indent=1)
print(json.dumps(res, indent=1))
