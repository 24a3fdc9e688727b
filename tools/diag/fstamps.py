"""Per-workgroup phases of the fused variable-length kernel on config 3
(diagnostic build with NVL_DIAG_FUSED): start, plan done, units done, counted."""
import ctypes, os, sys
import numpy as np, torch
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd()); sys.path.insert(0, R)
from nvlevelz_amd import _lib
import oracle, json
lib = ctypes.CDLL(os.path.abspath(os.environ.get("LIB", "build/libnvl_crc32c_fst.so")), mode=os.RTLD_LOCAL)
for name, (res, args) in _lib.SIGNATURES.items():
    f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
g = json.load(open(os.path.join(R, "tests", "golden", "configs.json")))["cfg3"]
if os.environ.get("CFG", "3") == "v":  # 10^5 x 4097 B at stride 4101
    lens = np.full(100_000, 4097, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(lens + 4)[:-1]]).astype(np.int64); n = lens.size
    g = dict(g, total=int(offs[-1] + lens[-1]) + 4, digest=None)
else:
    lens = oracle.port().cfg3_lengths(g["len_seed"], g["total"])
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64); n = lens.size
buf = torch.empty(g["total"] + 64, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), (g["total"] + 64) // 8, 8, 0, 1, g["seed"], None)
o = torch.from_numpy(offs).to(dev); m = torch.from_numpy(lens.astype(np.int64)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
wsb = lib.nvl_crc32c_batch_workspace_bytes(n); ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
for _ in range(5):
    assert lib.nvl_crc32c_batch_dev(buf.data_ptr(), o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n, 0, ws.data_ptr(), wsb, st) == 0
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
assert lib.nvl_crc32c_batch_dev(buf.data_ptr(), o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n, 0, ws.data_ptr(), wsb, st) == 0
e1.record()
torch.cuda.synchronize()
print("event us of the stamped launch:", e0.elapsed_time(e1) * 1e3)
h = np.zeros(8 * 1024, dtype=np.uint64)
lib.nvl_diag_fstamps.restype = ctypes.c_int
lib.nvl_diag_fstamps(h.ctypes.data_as(ctypes.c_void_p), h.size)
h = h.reshape(-1, 8).astype(np.int64)
h = h[h[:, 0] > 0]
last = h[h[:, 7] > 0]
print("last WG end (us after first start):", (last[:, 7] - h[:, 0].min()) / 100.0)
h[h[:, 7] == 0, 7] = h[h[:, 7] > 0, 7].max() if (h[:, 7] > 0).any() else 0
t0 = h[:, 0].min()
us = (h - t0) / 100.0
for k, name in enumerate(["start", "plan_done", "units_done", "counted", "4", "5", "6", "last_end"]):
    q = np.percentile(us[:, k], [0, 10, 50, 90, 100])
    print(f"{name:11s}", " ".join(f"{x:8.2f}" for x in q))
print("plan duration p50/max:", np.median(us[:, 1] - us[:, 0]), (us[:, 1] - us[:, 0]).max())
if g["digest"] is not None:
    print("digest ok:", oracle.port().digest(out.cpu().numpy().view(np.uint32)) == g["digest"])
