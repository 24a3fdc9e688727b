"""Per-wave timeline of one fast-path launch (diagnostic variant build: make -C nvlevelz_amd/csrc variant NAME=stamps VFLAGS_crc32c_fixed="-include ../../tools/diag/stamps.h")."""
import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_stamps.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
n, L = int(os.environ.get("N", "100000")), 4096
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
out = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, None, 0, st)
torch.cuda.synchronize()
h = np.zeros(4 * 4096, dtype=np.uint64)
lib.nvl_diag_stamps.restype = ctypes.c_int
lib.nvl_diag_stamps(h.ctypes.data_as(ctypes.c_void_p), h.size)
h = h.reshape(-1, 4).astype(np.int64)
t0 = h[:, 0].min()
start, fill, end = (h[:, 0] - t0), (h[:, 1] - t0), (h[:, 2] - t0)
xcc = h[:, 3] >> 32; cnt = h[:, 3] & 0xFFFFFFFF
# s_memrealtime: 100 MHz constant clock -> 10 ns ticks; report microseconds
start, fill, end = start / 100.0, fill / 100.0, end / 100.0
span = end.max()
print("span us", span)
for name, v in [("start", start), ("fill_done", fill), ("end", end), ("busy", end - fill)]:
    q = np.percentile(v, [0, 10, 50, 90, 100])
    print(f"{name:10s}", " ".join(f"{x:9.2f}" for x in q), " (% of span: " + " ".join(f"{100*x/span:5.1f}" for x in q) + ")")
for c in sorted(set(cnt.tolist())):
    m = cnt == c
    print(f"chunks={c:3d} waves={m.sum():5d} end p50={np.median(end[m])/span*100:5.1f}% max={end[m].max()/span*100:5.1f}% busy p50={np.median((end-fill)[m]):8.2f}us")
for x in range(8):
    m = xcc == x
    print(f"xcc {x}: waves {m.sum():4d} start p50 {np.median(start[m]):6.2f} max {start[m].max():6.2f} fill p50 {np.median(fill[m]):6.2f} end p50 {np.median(end[m]):6.2f} min {end[m].min():6.2f} max {end[m].max():6.2f}")
# per-workgroup view (16 waves per workgroup): spread inside a CU vs across CUs
wg = end.reshape(-1, 16)
wg_max, wg_min = wg.max(1), wg.min(1)
print("per-WG end spread (max-min) us p10/p50/p90:", " ".join(f"{x:.2f}" for x in np.percentile(wg_max - wg_min, [10, 50, 90])))
print("per-WG last-wave end us p0/p10/p50/p90/p100:", " ".join(f"{x:.2f}" for x in np.percentile(wg_max, [0, 10, 50, 90, 100])))
print("per-WG first-wave end us p0/p50/p100:", " ".join(f"{x:.2f}" for x in np.percentile(wg_min, [0, 50, 100])))
