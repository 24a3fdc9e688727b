"""Per-wave timeline of crc32c_head_kernel (diagnostic build with
-DNVL_DIAG_HSTAMPS): start, tables ready, end, and the cycles spent in the
long-head passes.  CFG=rand (10^5 buffers of 3364..4109 B) or CFG=3."""
import ctypes, json, os, sys
import numpy as np, torch
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd()); sys.path.insert(0, R)
from nvlevelz_amd import _lib
import oracle
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_hst.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    if hasattr(lib, name):
        f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
cfg = os.environ.get("CFG", "rand")
if cfg == "3":
    g = json.load(open(os.path.join(R, "tests", "golden", "configs.json")))["cfg3"]
    lens = oracle.port().cfg3_lengths(g["len_seed"], g["total"]).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    total, seed = g["total"], g["seed"]
else:
    n = 100_000
    lens = np.random.default_rng(7).integers(3364, 4110, n).astype(np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 4)[:-1]]).astype(np.int64)
    total, seed = int(offs[-1] + lens[-1]) + 4, 0x5EED0001
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
lib.nvl_diag_hstamps.restype = ctypes.c_int
assert lib.nvl_diag_hstamps(h.ctypes.data_as(ctypes.c_void_p), h.size) == 0
h = h.reshape(-1, 4).astype(np.int64)
h = h[h[:, 0] > 0]
t0 = h[:, 0].min()
us = lambda x: (x - t0) / 100.0  # s_memrealtime: 100 MHz
q = lambda v: " ".join(f"{x:8.2f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))
print(f"config {cfg}: waves {len(h)}")
print("start      ", q(us(h[:, 0])))
print("tables     ", q(us(h[:, 1])))
print("end        ", q(us(h[:, 2])))
print("long us    ", q(h[:, 3] / 100.0))
print("ok", int(out[0].item()) & 0xFFFFFFFF == oracle.port().value(buf[offs[0]:offs[0]+lens[0]].cpu().numpy().tobytes()) if hasattr(oracle.port(), "value") else "n/a")
