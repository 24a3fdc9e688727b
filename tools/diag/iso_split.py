"""Split one isolated config-2 launch: the stamps variant
build (tools/diag/stamps.h: per wave s_memrealtime at start, after the LDS
fill, at the end; 100 MHz) against the HIP events around the launch.
    make -C nvlevelz_amd/csrc variant NAME=stamps VFLAGS_crc32c_fixed="-include ../../tools/diag/stamps.h"
    LIB=build/libnvl_crc32c_stamps.so python tools/diag/iso_split.py [ITERS=30]
Per launch: event_us (ordinary events before/after, idle queue), span_us (first
wave start -> last wave end), outside = event - span (dispatch, completion and
event packets), start_spread (last - first wave start: the dispatch ramp),
fill_us (median per-wave start -> after-fill), end_p50 / end_max (from the
first wave start) and the slowest XCD."""
import ctypes, json, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_stamps.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(lib, name):
        f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
n, L = 100_000, 4096
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
out = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
lib.nvl_diag_stamps.restype = ctypes.c_int
NWV = int(os.environ.get("NWAVES", "4096"))  # waves of the launch (compact kernel: 512 x 12 or 16)
h = np.zeros(4 * NWV, dtype=np.uint64)
rows = []
wg_ends = []  # per launch: each workgroup's last-wave end minus the launch's mean
for it in range(int(os.environ.get("ITERS", "30"))):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, None, 0, st)
    e1.record()
    torch.cuda.synchronize()
    ev = e0.elapsed_time(e1) * 1e3
    lib.nvl_diag_stamps(h.ctypes.data_as(ctypes.c_void_p), h.size)
    s = h.reshape(-1, 4).astype(np.int64)[:NWV]
    t0 = s[:, 0].min()
    start = (s[:, 0] - t0) / 100.0
    fill = (s[:, 1] - s[:, 0]) / 100.0
    end = (s[:, 2] - t0) / 100.0
    xcc = s[:, 3] >> 32
    xend = [float(end[xcc == x].max()) for x in range(8)]
    r = {"event_us": round(ev, 2), "span_us": round(float(end.max()), 2),
         "outside_us": round(ev - float(end.max()), 2), "start_spread_us": round(float(start.max()), 2),
         "fill_us_p50": round(float(np.median(fill)), 2), "fill_us_max": round(float(fill.max()), 2),
         "end_p50_us": round(float(np.median(end)), 2), "end_max_us": round(float(end.max()), 2),
         "xcd_end_us": [round(x, 2) for x in xend]}
    cnt = (s[:, 3] & 0xFFFFFFFF).astype(np.float64)
    busy = (s[:, 2] - s[:, 1]) / 100.0
    r["units_p10_p50_p90"] = [float(np.percentile(cnt, q)) for q in (10, 50, 90)]
    wpg = int(os.environ.get("WAVES_PER_WG", "16"))
    wge = end[: (len(end) // wpg) * wpg].reshape(-1, wpg).max(axis=1)  # each workgroup's last wave end
    r["wg_end_mean_p10_p50_p90_max"] = [round(float(wge.mean()), 2)] + [round(float(np.percentile(wge, q)), 2)
                                                                         for q in (10, 50, 90, 100)]
    wg_ends.append(wge - wge.mean())  # each workgroup's lateness in this launch
    r["units_total"] = int(cnt.sum())
    r["us_per_unit_p50"] = round(float(np.median(busy / np.maximum(cnt, 1))), 3)
    rows.append(r)
    print(json.dumps(r), flush=True)
keys = ["event_us", "span_us", "outside_us", "start_spread_us", "fill_us_p50", "end_p50_us", "end_max_us"]
if len(wg_ends) > 4:  # is a workgroup's lateness persistent from one launch to the next?
    W = np.array(wg_ends[2:])
    cc = [float(np.corrcoef(W[k], W[k + 1])[0, 1]) for k in range(len(W) - 1)]
    mean_late = W.mean(axis=0)
    print(json.dumps({"wg_lateness_corr_consecutive_launches": [round(c, 3) for c in cc[:8]],
                      "corr_median": round(float(np.median(cc)), 3),
                      "std_per_launch_us": round(float(W.std(axis=1).mean()), 2),
                      "std_of_mean_over_launches_us": round(float(mean_late.std()), 2)}))
print(json.dumps({"wg_end_median_of_launches": [round(float(np.median([r["wg_end_mean_p10_p50_p90_max"][k] for r in rows[2:]])), 2)
                                                for k in range(5)]}))
print(json.dumps({"median": {k: round(float(np.median([r[k] for r in rows[2:]])), 2) for k in keys}}))
