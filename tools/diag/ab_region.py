"""Interleaved timing of library variants on the region path (one process):
    python tools/diag/ab_region.py CONFIG lib_A.so lib_B.so ...   (CONFIG: vR, rR, 3R, uR, uoR)
M rounds x R back-to-back calls per variant, HIP events around each round
(mean per call = the sustained period) and around single calls (median)."""
import ctypes, json, os, sys
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib


def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            f = getattr(lib, name); f.restype = res; f.argtypes = args
    return lib


cfg, paths = sys.argv[1], sys.argv[2:]
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
libs = [load(p) for p in paths]
for lib in libs:
    assert lib.nvl_crc32c_init(0) == 0
import oracle
if cfg == "3R":
    lens = oracle.port().cfg3_lengths(0x5EED0003, 1 << 30).astype(np.int64); gap = 0; total = 1 << 30
    alg = total + 12 * lens.size
else:
    lens = (np.full(100_000, 4097) if cfg == "vR" else np.random.default_rng(7).integers(3364, 4110, 100_000)
            ).astype(np.int64); gap = 4
    total = int((lens + gap).sum()); alg = int(lens.sum()) + 20 * lens.size
offs = np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64)
if cfg in ("uR", "uoR"):  # 10^5 x 4096 B shuffled (not region-shaped: the page path), uoR from an odd base
    lens = np.full(100_000, 4096, dtype=np.int64)
    offs = (4096 * np.random.default_rng(1).permutation(lens.size) + (3 if cfg == "uoR" else 0)).astype(np.int64)
    total = int(offs.max()) + 4096; alg = int(lens.sum()) + 20 * lens.size
n = lens.size
buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
libs[0].nvl_crc32c_fill_splitmix(buf.data_ptr(), (total + 64) // 8, 8, 0, 1, 0x5EED00B1, None)
o = torch.from_numpy(offs).to(dev); m = torch.from_numpy(lens).to(dev)
outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in libs]
wsb = max(lib.nvl_crc32c_region_workspace_bytes(total, n) for lib in libs)  # (variants may need more)
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
# NVL_CRC32C_FLAG_REGION_SHAPED by default: the region kernel alone (AB_FLAGS=0: the routed call)
FLAGS = int(os.environ.get("AB_FLAGS", "2"))
nfix = 100_000  # the config-2 reference (fixed path, first library) timed in the same rounds
fbuf = torch.empty(nfix * 4096, dtype=torch.uint8, device=dev)
libs[0].nvl_crc32c_fill_splitmix(fbuf.data_ptr(), nfix, 4096, 0, 1, 0x5EED0001, None)
fout = torch.empty(nfix, dtype=torch.int32, device=dev)


def run(k):
    if k == len(libs):
        return libs[0].nvl_crc32c_fixed_dev(fbuf.data_ptr(), 4096, 4096, nfix, None, 0, fout.data_ptr(), 0, None, 0,
                                            st)
    return libs[k].nvl_crc32c_region_dev(buf.data_ptr(), total, o.data_ptr(), m.data_ptr(), None, 0,
                                         outs[k].data_ptr(), n, FLAGS, ws.data_ptr(), wsb, st)
rounds, reps = int(os.environ.get("AB_ROUNDS", "10")), int(os.environ.get("AB_REPS", "30"))
per = [[] for _ in range(len(libs) + 1)]
single = [[] for _ in range(len(libs) + 1)]
for k in range(len(libs) + 1):
    for _ in range(5):
        rc = run(k)
        assert rc == 0, (k, rc)
torch.cuda.synchronize()
import time
t0 = time.perf_counter()  # ~100 ms of load first: the GPU's sustained-load state (the first ~30 ms run slower)
while time.perf_counter() - t0 < 0.1:
    for k in range(len(libs) + 1):
        for _ in range(5): run(k)
    torch.cuda.synchronize()
for r in range(rounds):
    ks = list(range(len(libs) + 1))
    for k in ks[r % len(ks):] + ks[:r % len(ks)]:  # (rotated each round: no variant always follows the same one)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps): run(k)
        e1.record()
        torch.cuda.synchronize()
        per[k].append(e0.elapsed_time(e1) * 1e3 / reps)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(10)]
        for j in range(5):
            ev[2 * j].record(); run(k); ev[2 * j + 1].record()
        torch.cuda.synchronize()
        single[k] += [ev[2 * j].elapsed_time(ev[2 * j + 1]) * 1e3 for j in range(5)]
ref = outs[0].cpu()
t = float(np.median(per[-1]))
print(json.dumps({"config": "cfg2 (fixed path, first library)", "period_us": round(t, 2),
                  "period_rounds": [round(x, 1) for x in per[-1]], "frac": round(100_000 * 4100 / (t * 1e-6) / 8e12, 4)}),
      flush=True)
for k, p in enumerate(paths):
    t = float(np.median(per[k]))
    print(json.dumps({"config": cfg, "variant": os.path.basename(p), "period_us": round(t, 2),
                      "period_rounds": [round(x, 1) for x in per[k]], "single_median_us": round(float(np.median(single[k])), 2),
                      "frac": round(alg / (t * 1e-6) / 8e12, 4), "same_as_first": bool(torch.equal(outs[k].cpu(), ref))}),
          flush=True)
