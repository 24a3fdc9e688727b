"""Sustained-rate evidence: K back-to-back launches of a
workload with an event every SEG launches, while a thread samples the GPU's
own metrics (amdsmi gpu_metrics: gfx clock, memory clock, socket power,
temperature, throttle status) -- does the launch period drift with the clock?
    python tools/diag/clocks.py [--config cfg2|cfg3R|vR] [--launches 2000] [--seg 50]
One JSON line per segment: launches, mean period (us) and the metrics sampled
during it (mean), then a summary line."""
import argparse, json, os, sys, threading, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))))
import torch
from nvlevelz_amd import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="cfg2")
ap.add_argument("--launches", type=int, default=2000)
ap.add_argument("--seg", type=int, default=50)
ap.add_argument("--idle-ms", type=float, default=0.0, help="sleep before the run (cool-down)")
a = ap.parse_args()
lib = _lib.lib
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
st = torch.cuda.current_stream().cuda_stream

# --- the workload ------------------------------------------------------------
if a.config == "cfg2":
    n, L = 100_000, 4096
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    bp, op = buf.data_ptr(), out.data_ptr()
    step = lambda: lib.nvl_crc32c_fixed_dev(bp, L, L, n, None, 0, op, 0, None, 0, st)
    alg = n * (L + 4)
else:
    import oracle
    if a.config == "cfg3R":
        lens = oracle.port().cfg3_lengths(0x5EED0003, 1 << 30).astype(np.int64)
        total = 1 << 30
        alg = total + 12 * lens.size
    else:  # vR
        lens = np.full(100_000, 4097, dtype=np.int64)
        total = int((lens + 4).sum())
        alg = int(lens.sum()) + 20 * lens.size
    offs = np.concatenate([[0], np.cumsum(lens + (0 if a.config == "cfg3R" else 4))[:-1]]).astype(np.int64)
    buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), (total + 64) // 8, 8, 0, 1, 0x5EED0002, None)
    o = torch.from_numpy(offs).to(dev)
    m = torch.from_numpy(lens).to(dev)
    n = lens.size
    out = torch.empty(n, dtype=torch.int32, device=dev)
    wsb = lib.nvl_crc32c_region_workspace_bytes(total, n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    step = lambda: lib.nvl_crc32c_region_dev(buf.data_ptr(), total, o.data_ptr(), m.data_ptr(), None, 0,
                                             out.data_ptr(), n, 0, ws.data_ptr(), wsb, st)

# --- metrics sampler -----------------------------------------------------------
samples, stop = [], threading.Event()
KEYS = None
try:
    import amdsmi
    amdsmi.amdsmi_init()
    hs = amdsmi.amdsmi_get_processor_handles()
    bus = torch.cuda.get_device_properties(0).pci_bus_id if hasattr(torch.cuda.get_device_properties(0),
                                                                   "pci_bus_id") else None
    h = hs[0]
    for x in hs:
        try:
            bdf = amdsmi.amdsmi_get_gpu_device_bdf(x)
            if bus is not None and int(bdf.split(":")[1], 16) == bus:
                h = x
        except Exception:  # noqa: BLE001
            pass

    def read():
        mtr = amdsmi.amdsmi_get_gpu_metrics_info(h)
        d = {}
        for k, v in mtr.items():
            if isinstance(v, (int, float)) and v not in (65535, 0xFFFFFFFF, 0xFFFFFFFFFFFFFFFF):
                d[k] = v
            elif isinstance(v, list):
                vals = [x for x in v if isinstance(x, (int, float)) and x not in (65535, 0xFFFFFFFF)]
                if vals:
                    d[k] = float(np.mean(vals))
        return d
    read()
    metrics_ok = True
except Exception as e:  # noqa: BLE001 -- the box may not expose gpu_metrics to the user
    metrics_ok = repr(e)


def sampler():
    while not stop.is_set():
        try:
            samples.append((time.perf_counter(), read()))
        except Exception:  # noqa: BLE001
            pass
        time.sleep(0.001)


for _ in range(20):
    step()
torch.cuda.synchronize()
if a.idle_ms:
    time.sleep(a.idle_ms / 1e3)
th = threading.Thread(target=sampler, daemon=True)
if metrics_ok is True:
    th.start()
    time.sleep(0.01)
nseg = a.launches // a.seg
ev = [torch.cuda.Event(enable_timing=True) for _ in range(nseg + 1)]
t_host = [0.0] * (nseg + 1)
t_host[0] = time.perf_counter()
ev[0].record()
for j in range(nseg):
    for _ in range(a.seg):
        step()
    ev[j + 1].record()
torch.cuda.synchronize()
t_end = time.perf_counter()
stop.set()
if metrics_ok is True:
    th.join()
per = [ev[j].elapsed_time(ev[j + 1]) * 1e3 / a.seg for j in range(nseg)]
# segment j's GPU time window, mapped onto the host clock: the GPU ran the
# segments back to back from (t_end - total) on
tot = sum(per) * a.seg * 1e-6
t0 = t_end - tot
edges = np.concatenate([[0.0], np.cumsum(np.array(per) * a.seg * 1e-6)]) + t0
rows = []
for j in range(nseg):
    ss = [d for (t, d) in samples if edges[j] <= t < edges[j + 1]]
    mean = {}
    for k in (ss[0].keys() if ss else []):
        vals = [d[k] for d in ss if k in d]
        mean[k] = round(float(np.mean(vals)), 1)
    r = {"segment": j, "launches": a.seg, "period_us": round(per[j], 2),
         "frac": round(alg / (per[j] * 1e-6) / 8e12, 4), "samples": len(ss), "metrics": mean}
    rows.append(r)
    print(json.dumps(r), flush=True)
print(json.dumps({"config": a.config, "launches": nseg * a.seg, "first_period_us": round(per[0], 2),
                  "last_period_us": round(per[-1], 2), "mean_period_us": round(float(np.mean(per)), 2),
                  "metrics_available": metrics_ok}))
