"""Phase timeline of the head kernel (run_heads) on a variable-length batch,
from a diagnostic variant build with tools/diag/stamps.h force-included:
    make -C nvlevelz_amd/csrc variant NAME=stamps VFLAGS_crc32c_region="-include ../../tools/diag/stamps.h"
    CFG=r|v|3|u LIB=build/libnvl_crc32c_stamps.so python tools/diag/tl.py
(r, v, 3 are region-shaped and batch_dev now routes them to the region path;
u -- shuffled aligned 4 KiB -- keeps the head kernel's work, in the route kernel)
Stamps per wave (s_memrealtime, 100 MHz): 0 entry, 1 after the tile scan,
2 tables in LDS, 3 rounds done (last sub-range), 4 list barrier passed,
5 long-head drain done, 7 exit.  Prints percentiles of each phase (us) and
of the kernel span as seen from the earliest entry."""
import ctypes, os, sys
import numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path.insert(0, ROOT)
from nvlevelz_amd import _lib
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_stamps.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(lib, name):
        f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
cfg = os.environ.get("CFG", "r")
if cfg == "3":
    import oracle
    lens = oracle.port().cfg3_lengths(0x5EED0003, 1 << 30).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
elif cfg == "u":  # 10^5 aligned 4 KiB buffers in random order: not region-shaped, the route kernel runs the heads
    n = 100_000
    lens = np.full(n, 4096, dtype=np.int64)
    offs = np.random.default_rng(3).permutation(n).astype(np.int64) * 4096
else:
    n = 100_000
    lens = np.full(n, 4097, dtype=np.int64) if cfg == "v" else np.random.default_rng(7).integers(3364, 4110, n).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 4)[:-1]])
n = lens.size
total = int((offs + lens).max()) + 64
buf = torch.empty(total, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), total // 8, 8, 0, 1, 0x5EED00B1, None)
o = torch.from_numpy(offs).to(dev); m = torch.from_numpy(lens).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
wsb = lib.nvl_crc32c_batch_workspace_bytes(n)
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
for _ in range(6):
    lib.nvl_crc32c_batch_dev(buf.data_ptr(), o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n, 0,
                             ws.data_ptr(), wsb, st)
torch.cuda.synchronize()
h = np.zeros(8 * 65536, dtype=np.uint64)
lib.nvl_diag_tl.restype = ctypes.c_int
lib.nvl_diag_tl(h.ctypes.data_as(ctypes.c_void_p), h.size)
h = h.reshape(-1, 8).astype(np.int64)
h = h[h[:, 0] > 0]
t0 = h[:, 0].min()
rel = (h - t0) / 100.0
rel[h == 0] = np.nan
print(f"config {cfg}: n {n}, waves {len(h)}, span {np.nanmax(rel[:, 7]):.2f} us")
# stamp order in time: 0 entry, 2 fill issued (barrier passed unless the
# scan is fused), 1 fused tile scan done (its barrier), 3 lists complete,
# 4 own rounds done, 5 drain done, 7 exit
phases = [("fill", 0, 2), ("scan", 2, 1), ("classify", 1, 3), ("rounds", 3, 4), ("drain", 4, 5), ("to_exit", 5, 7)]
for name, a_, b_ in phases:
    d = rel[:, b_] - rel[:, a_]
    d = d[~np.isnan(d)]
    if d.size:
        q = np.percentile(d, [0, 10, 50, 90, 100])
        print(f"{name:13s} " + " ".join(f"{x:8.2f}" for x in q))
for k in (0, 3, 5, 7):
    v = rel[:, k]
    v = v[~np.isnan(v)]
    if v.size:
        q = np.percentile(v, [0, 10, 50, 90, 100])
        print(f"abs t{k:<10d} " + " ".join(f"{x:8.2f}" for x in q))

# per-workgroup end (16 waves each) by blockIdx % 8 (the XCD under round-robin placement)
end = rel[:, 7]
nw = len(end) // 16 * 16
wg_end = np.nanmax(end[:nw].reshape(-1, 16), axis=1)
wg_start = np.nanmin(rel[:nw, 0].reshape(-1, 16), axis=1)
print("per-WG end p0/p10/p50/p90/p100:", " ".join(f"{x:.2f}" for x in np.percentile(wg_end, [0, 10, 50, 90, 100])))
for x in range(8):
    e = wg_end[x::8]
    print(f"  b%8={x}: end p10 {np.percentile(e, 10):6.2f} p50 {np.median(e):6.2f} max {e.max():6.2f}  start p50 {np.median(wg_start[x::8]):5.2f}")
order = np.argsort(wg_end)
print("slowest WGs:", order[-8:].tolist(), "fastest:", order[:8].tolist())
