"""Summarise tools/diag/pmc_calib.sh: per kernel (and dispatch order for the
micro kernels), the raw counters per dispatch (no wave scaling), and for the
micro kernels their counted bytes over the known 1 GiB:
  fetch_x2 = FETCH_SIZE kB x 1024 x 2; req_bytes = 64 x (RDREQ + RDREQ_128B);
  tcc_req_bytes = 128 x TCC_REQ (L2 requests, any source)."""
import csv, glob, json, os, sys
from collections import defaultdict

d = sys.argv[1]
GiB = float(1 << 30)
out = {}
for part in ("micro", "cfg3s"):
    rows = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [per dispatch]
    order = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, part, "*counter_collection.csv"))):
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            names[k] = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]))
        for k in sorted(per, key=int):
            nm = names[k][0]
            for c, v in per[k].items():
                rows[nm][c].append(v)
            rows[nm]["grid_waves"].append(names[k][1] / 64)
    res = {}
    for nm, cs in rows.items():
        res[nm] = {c: [round(x) for x in v] for c, v in cs.items()}
    out[part] = res
# micro: dispatch sequence per rep = s16c(flush), s16nt, s16c, s4nt, s4nt(+4), s4c, s16mis
m = out.get("micro", {})
cal = {}
def pick(name, idx):
    return {c: v[idx] for c, v in m.get(name, {}).items() if idx < len(v)}
seq = {"s16nt": ("s16nt", 0), "s16c": ("s16c", 1), "s4nt": ("s4nt", 0), "s4nt4": ("s4nt", 1), "s4c": ("s4c", 0),
       "s16mis": ("s16mis", 0)}
for label, (nm, i) in seq.items():
    # s16c dispatches alternate flush / measured: the measured one is every second
    c = pick(nm, 2 if nm == "s16c" else i)  # s16c: flush, flush, measured, ... in dispatch order
    e = {}
    if "FETCH_SIZE" in c:
        e["fetch_x2_over_bytes"] = round(c["FETCH_SIZE"] * 1024 * 2 / GiB, 4)
    if "TCC_EA0_RDREQ_sum" in c:
        e["req_bytes_over_bytes"] = round(64 * (c["TCC_EA0_RDREQ_sum"] + c.get("TCC_EA0_RDREQ_128B_sum", 0)) / GiB, 4)
        e["rdreq_128B_share"] = round(c.get("TCC_EA0_RDREQ_128B_sum", 0) / max(c["TCC_EA0_RDREQ_sum"], 1), 4)
    if "TCC_REQ_sum" in c:
        e["tcc_req_x128_over_bytes"] = round(128 * c["TCC_REQ_sum"] / GiB, 4)
        e["tcc_hit_rate"] = round(c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1), 4)
        e["tcc_miss_x128_over_bytes"] = round(128 * c["TCC_MISS_sum"] / GiB, 4)
    if "TCP_TCC_READ_REQ_sum" in c:
        e["tcp_tcc_read_req_x128_over_bytes"] = round(128 * c["TCP_TCC_READ_REQ_sum"] / GiB, 4)
        e["tcp_tcc_read_req_x64_over_bytes"] = round(64 * c["TCP_TCC_READ_REQ_sum"] / GiB, 4)
    cal[label] = e
out["micro_calibration"] = cal
print(json.dumps(out, indent=1))
