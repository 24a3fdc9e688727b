"""Per-wave timeline of scheduler C (run_bufs) on a variable-length batch
(diagnostic variant build: make -C nvlevelz_amd/csrc variant NAME=stamps VFLAGS_crc32c_batch="-include ../../tools/diag/stamps.h"): start, after the LDS fill, end and
chunks walked per wave.  CFG=v (10^5 x 4097 B, unfused plan) or CFG=3 (config 3,
fused kernel)."""
import ctypes, json, os, sys
import numpy as np, torch
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd()); sys.path.insert(0, R)
from nvlevelz_amd import _lib
import oracle
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_bst.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(lib, name):
        f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
cfg = os.environ.get("CFG", "v")
p = oracle.port()
if cfg == "3":
    g = json.load(open(os.path.join(R, "tests", "golden", "configs.json")))["cfg3"]
    lens = p.cfg3_lengths(g["len_seed"], g["total"]).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    total, seed = g["total"], g["seed"]
else:
    n = 100_000
    lens = np.full(n, 4097, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 4)[:-1]]).astype(np.int64)
    total, seed = int(offs[-1] + lens[-1]) + 4, 0x5EED00B1
n = lens.size
buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), (total + 64) // 8, 8, 0, 1, seed, None)
o = torch.from_numpy(offs).to(dev); m = torch.from_numpy(lens).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
wsb = lib.nvl_crc32c_batch_workspace_bytes(n); ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
call = lambda: lib.nvl_crc32c_batch_dev(buf.data_ptr(), o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n, 0,
                                        ws.data_ptr(), wsb, st)
for _ in range(5):
    assert call() == 0
torch.cuda.synchronize()
h = np.zeros(4 * 4096, dtype=np.uint64)
lib.nvl_diag_stamps(h.ctypes.data_as(ctypes.c_void_p), h.size)
h = h.reshape(-1, 4).astype(np.int64)
h = h[h[:, 0] > 0]
t0 = h[:, 0].min()
start, fill, end = (h[:, 0] - t0) / 100.0, (h[:, 1] - t0) / 100.0, (h[:, 2] - t0) / 100.0
cnt = h[:, 3] & 0xFFFFFFFF
span = end.max()
print(f"config {cfg}: waves {len(h)} span {span:.2f} us, chunk steps total {cnt.sum()}")
for name, v in [("start", start), ("fill_done", fill), ("end", end), ("busy", end - fill)]:
    q = np.percentile(v, [0, 10, 50, 90, 100])
    print(f"{name:10s}", " ".join(f"{x:9.2f}" for x in q))
q = np.percentile(cnt, [0, 10, 50, 90, 100])
print("steps/wave", " ".join(f"{x:9.1f}" for x in q))
busy = end - fill
rate = busy[cnt > 0] / cnt[cnt > 0]
print("us per step p10/p50/p90:", " ".join(f"{x:.3f}" for x in np.percentile(rate, [10, 50, 90])))
wg = end.reshape(-1, 16)
print("per-WG end spread (max-min) us p10/p50/p90:", " ".join(f"{x:.2f}" for x in np.percentile(wg.max(1) - wg.min(1), [10, 50, 90])))
print("per-WG last end us p0/p10/p50/p90/p100:", " ".join(f"{x:.2f}" for x in np.percentile(wg.max(1), [0, 10, 50, 90, 100])))
wc = cnt.reshape(-1, 16).sum(1)
print("per-WG steps p0/p50/p100:", " ".join(f"{x:.0f}" for x in np.percentile(wc, [0, 50, 100])))
