"""Per-XCD end times of consecutive config-2 launches (stamps variant build,
see tools/diag/stamps.py): is the slowest XCD the same launch after launch?
    LIB=build/libnvl_crc32c_stamps.so python tools/diag/stamps_xcd.py"""
import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_stamps.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
n, L = 100_000, 4096
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
out = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
lib.nvl_diag_stamps.restype = ctypes.c_int
h = np.zeros(4 * 4096, dtype=np.uint64)
rows = []
for it in range(int(os.environ.get("ITERS", "12"))):
    for _ in range(int(os.environ.get("BACK", "1"))):  # back-to-back launches; the last one's stamps are kept
        lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, None, 0, st)
    torch.cuda.synchronize()
    lib.nvl_diag_stamps(h.ctypes.data_as(ctypes.c_void_p), h.size)
    s = h.reshape(-1, 4).astype(np.int64)
    t0 = s[:, 0].min()
    end = (s[:, 2] - t0) / 100.0
    xcc = s[:, 3] >> 32
    wg = np.arange(end.size) // 16
    if it == 0:
        print("waves with XCC id == workgroup % 8:", float(np.mean(xcc == wg % 8)), flush=True)
    med = [float(np.median(end[xcc == x])) for x in range(8)]
    mx = [float(end[xcc == x].max()) for x in range(8)]
    rows.append(med)
    print(f"launch {it:2d} span {end.max():6.2f}  XCD end p50: " + " ".join(f"{m:6.2f}" for m in med)
          + "  max: " + " ".join(f"{m:6.2f}" for m in mx), flush=True)
r = np.array(rows)
rank = np.argsort(np.argsort(-r, axis=1), axis=1)  # 0 = slowest
print("mean p50 per XCD:", " ".join(f"{x:6.2f}" for x in r.mean(0)))
print("std  p50 per XCD:", " ".join(f"{x:6.2f}" for x in r.std(0)))
print("slowest-rank counts (rank 0 = slowest) per XCD:", [int((rank[:, x] == 0).sum()) for x in range(8)])
