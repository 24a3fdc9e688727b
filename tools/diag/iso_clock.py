"""Isolated vs back-to-back config-2 launches with per-wave shader clocks
(VERDICT r05 item 6).  The stamps_clk variant build records, per wave, its
start / after-fill / end (s_memrealtime, 100 MHz) and s_memtime at start and
end: a wave's average shader clock = d(memtime) / d(memrealtime) x 100 MHz.
    make -C nvlevelz_amd/csrc variant NAME=stampsclk VFLAGS_crc32c_fixed="-include ../../tools/diag/stamps_clk.h"
    LIB=build/libnvl_crc32c_stampsclk.so python tools/diag/iso_clock.py
Modes, each ITERS launches, the stamps of every launch read back:
  isolated  -- synchronize before each launch (an idle queue, a shim call)
  queued    -- back to back (the bench's timed region): the stamps of each
               launch are read after a run of 8 launches (the last one's)
Per mode: median over launches of the launch span, median wave clock (MHz),
fill (start -> after fill), per-unit time, end spread."""
import ctypes, json, os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_stampsclk.so")), mode=os.RTLD_LOCAL)
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
NWV = 4096
h = np.zeros(8 * 65536, dtype=np.uint64)


def launch():
    assert lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, None, 0, st) == 0


def one(mode):
    if mode == "isolated":
        torch.cuda.synchronize()
        time.sleep(0.0005)  # a host round trip's idle gap, as a synchronous caller leaves
        launch()
    else:
        for _ in range(8):
            launch()
    torch.cuda.synchronize()
    lib.nvl_diag_stamps8(h.ctypes.data_as(ctypes.c_void_p), h.size)
    s = h.reshape(-1, 8).astype(np.int64)[:NWV]
    t0 = s[:, 0].min()
    dt = np.maximum(s[:, 2] - s[:, 0], 1)
    clk = (s[:, 5] - s[:, 4]) / dt * 100.0  # MHz
    cnt = np.maximum((s[:, 3] & 0xFFFFFFFF).astype(np.float64), 1)
    end = (s[:, 2] - t0) / 100.0
    wstart = ((s[:, 0] - t0) / 100.0).reshape(-1, 16).min(axis=1)  # each workgroup's first wave start
    wend = end.reshape(-1, 16).max(axis=1)
    one.starts.append(wstart)
    one.ends.append(wend)
    return {"span_us": float(end.max()), "clock_mhz_p50": float(np.median(clk)), "clock_mhz_p10": float(np.percentile(clk, 10)),
            "fill_us_p50": float(np.median((s[:, 1] - s[:, 0]) / 100.0)),
            "us_per_unit_p50": float(np.median((s[:, 2] - s[:, 1]) / 100.0 / cnt)),
            "end_p50_us": float(np.median(end)), "start_spread_us": float((s[:, 0].max() - t0) / 100.0)}


one.starts, one.ends = [], []
launch(); torch.cuda.synchronize()
for _ in range(300):  # the sustained state first
    launch()
res = {}
for mode in ("queued", "isolated", "queued", "isolated"):
    one.starts, one.ends = [], []
    rows = [one(mode) for _ in range(int(os.environ.get("ITERS", "20")))]
    r = {k: round(float(np.median([x[k] for x in rows])), 2) for k in rows[0]}
    st_ = np.median(np.array(one.starts), axis=0)
    en_ = np.median(np.array(one.ends), axis=0)
    r["wg_start_us_by_id_32"] = [round(float(x), 2) for x in st_.reshape(-1, 32).mean(axis=1)]
    r["wg_end_us_by_id_32"] = [round(float(x), 2) for x in en_.reshape(-1, 32).mean(axis=1)]
    r["wg_start_vs_id_slope_us"] = round(float(np.polyfit(np.arange(st_.size) / st_.size, st_, 1)[0]), 2)
    res.setdefault(mode, []).append(r)
print(json.dumps(res))
