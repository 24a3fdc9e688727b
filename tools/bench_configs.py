"""Time BASELINE configs and the call-site shapes through the C ABI (HIP events
around each call, median of R reps), every result checked.
    python tools/bench_configs.py [--lib build/libnvl_crc32c_X.so] [--configs 2,3,4,v,g,r]
  2, 3, 4  BASELINE configs 2-4 (golden digests)
  3R, vR, rR  config 3, v and r through nvl_crc32c_region_dev (layout checked on the device: plan,
           region path, the body kernel's early exit)
  3S, vS, rS  the same with NVL_CRC32C_FLAG_REGION_SHAPED (the region kernel alone, one launch)
  u, uR    10^5 x 4 KiB at 4 KiB-aligned offsets in a random order (not region-shaped) through
           nvl_crc32c_batch_dev / nvl_crc32c_region_dev (both: plan, then the page path)
  uo       u from an odd base (the page path's realigned passes), nvl_crc32c_batch_dev
  big1     one aligned 1 GiB buffer (fixed path, n = 1)
  v        10^5 x 4097 B at stride 4101: block | type of 4096-byte SSTable blocks with their
           4-byte stored CRC between them (whole-table verify shape), nvl_crc32c_batch_dev
  g        10^5 x 4096 B at stride 4099 from an odd base: the fixed-stride general path
  f        10^5 x 3500 B at stride 4128 from base 48: fixed-stride one-partial-chunk buffers
  q        10^5 x 3500 B packed at stride 3500: the same, some starts in a page's first granule
  r        10^5 buffers of 3364..4109 B (the n+1 of data blocks at block_size 4096)
           at stride length+4, nvl_crc32c_batch_dev
  3, v and r through nvl_crc32c_batch_dev are region-shaped: routed to the region path.
v, g, r and u are checked CRC by CRC against the oracle."""
import argparse, time, ctypes, json, os, sys
import numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from nvlevelz_amd import _lib
import oracle
ap = argparse.ArgumentParser(); ap.add_argument("--lib"); ap.add_argument("--configs", default="2,3,4")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--warm-ms", type=float, default=60.0)
a = ap.parse_args()
lib = _lib.lib
if a.lib:
    lib = ctypes.CDLL(os.path.abspath(a.lib), mode=os.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        if not hasattr(lib, name):  # older variant builds lack newer entry points
            continue
        f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
st = torch.cuda.current_stream().cuda_stream
g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
p = oracle.port()


SUSTAINED = {}


def timeit(fn, reps):
    """Median of single calls (events around each), after a warm-up of
    a.warm_ms of back-to-back calls (the GPU's sustained-load state: the
    first ~30 ms of load run ~15 % slower, profiles/r04_clocks_cfg2.jsonl);
    also the sustained period of reps back-to-back calls (SUSTAINED)."""
    t0 = time.perf_counter()
    while True:
        for _ in range(10): fn()
        torch.cuda.synchronize()
        if time.perf_counter() - t0 > a.warm_ms * 1e-3:
            break
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
    for j in range(reps):
        ev[2*j].record(); fn(); ev[2*j+1].record()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record()
    torch.cuda.synchronize()
    SUSTAINED["period"] = e0.elapsed_time(e1) * 1e-3 / reps
    return float(np.median([ev[2*j].elapsed_time(ev[2*j+1]) for j in range(reps)])) * 1e-3


def varlen(offs, lens, total, seed, region=False, shaped=False):
    n = lens.size
    buf = torch.empty(total + 64, dtype=torch.uint8, device=dev)
    lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), (total + 64) // 8, 8, 0, 1, seed, None)
    o = torch.from_numpy(offs.astype(np.int64)).to(dev); m = torch.from_numpy(lens.astype(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    if region:  # nvl_crc32c_region_dev over the region [buf, buf + total)
        wsb = lib.nvl_crc32c_region_workspace_bytes(total, n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        fl = _lib.FLAG_REGION_SHAPED if shaped else 0
        fn = lambda: lib.nvl_crc32c_region_dev(buf.data_ptr(), total, o.data_ptr(), m.data_ptr(), None, 0,
                                               out.data_ptr(), n, fl, ws.data_ptr(), wsb, st)
        return buf, out, fn, (o, m, ws)
    wsb = lib.nvl_crc32c_batch_workspace_bytes(n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    fn = lambda: lib.nvl_crc32c_batch_dev(buf.data_ptr(), o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n, 0,
                                          ws.data_ptr(), wsb, st)
    return buf, out, fn, (o, m, ws)


for c in a.configs.split(","):
    keep = None
    if c in ("2", "4"):
        cfg = g[f"cfg{c}"]; n, L = cfg["n"], cfg["len"]
        buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
        lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, cfg["seed"], None)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        wsb = max(1, lib.nvl_crc32c_fixed_workspace_bytes(L, L, n))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        fn = lambda: lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, ws.data_ptr(), wsb, st)
        alg = n * (L + 4)
        check = lambda res: p.digest(res) == cfg["digest"]
    elif c == "big1":  # one aligned 1 GiB buffer (a lone huge fixed batch: scheduler B, not the chunk fold)
        n, L = 1, 1 << 30
        buf = torch.empty(L, dtype=torch.uint8, device=dev)
        lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), L // 8, 8, 0, 1, 0x5EED0B16, None)
        out = torch.empty(1, dtype=torch.int32, device=dev)
        wsb = max(1, lib.nvl_crc32c_fixed_workspace_bytes(L, L, 1))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        fn = lambda: lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, 1, None, 0, out.data_ptr(), 0, ws.data_ptr(), wsb, st)
        alg = L + 4
        want = p.fixed(buf.cpu().numpy(), L, L, 1)
        check = lambda res: bool(np.array_equal(res, want))
    elif c in ("3", "3R", "3S"):
        cfg = g["cfg3"]; total = cfg["total"]
        lens = p.cfg3_lengths(cfg["len_seed"], total)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]])
        n = lens.size
        buf, out, fn, keep = varlen(offs, lens, total, cfg["seed"], region=c != "3", shaped=c == "3S")
        alg = total + 12 * n
        check = lambda res: p.digest(res) == cfg["digest"]
    elif c == "rs":  # r's lengths packed in a shuffled order: not sorted, so batch_dev runs the batch kernels
        n = 100_000
        lens = np.random.default_rng(7).integers(3364, 4110, n).astype(np.int64)
        perm = np.random.default_rng(9).permutation(n)
        slot = np.concatenate([[0], np.cumsum(lens[perm] + 4)[:-1]])
        offs = np.empty(n, dtype=np.int64)
        offs[perm] = slot
        total = int(slot[-1] + lens[perm[-1]]) + 4
        buf, out, fn, keep = varlen(offs, lens, total, 0x5EED00B1)
        alg = int(lens.sum()) + 20 * n
        host = buf.cpu().numpy()
        check = lambda res: bool(np.array_equal(res, p.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64))))
    elif c in ("v", "r", "vR", "rR", "vS", "rS", "u", "uR", "uo"):
        n = 100_000
        if c[0] == "v":
            lens = np.full(n, 4097, dtype=np.int64)
        elif c[0] == "u":
            lens = np.full(n, 4096, dtype=np.int64)
        else:
            lens = np.random.default_rng(7).integers(3364, 4110, n).astype(np.int64)
        if c[0] == "u":
            offs = np.random.default_rng(8).permutation(n).astype(np.int64) * 4096 + (3 if c == "uo" else 0)
            total = n * 4096 + (3 if c == "uo" else 0)
        else:
            offs = np.concatenate([[0], np.cumsum(lens + 4)[:-1]])
            total = int(offs[-1] + lens[-1]) + 4
        buf, out, fn, keep = varlen(offs, lens, total, 0x5EED00B1, region=c[1:] in ("R", "S"), shaped=c[1:] == "S")
        alg = int(lens.sum()) + 20 * n
        host = buf.cpu().numpy()
        check = lambda res: bool(np.array_equal(res, p.varlen(host, offs.astype(np.uint64), lens.astype(np.uint64))))
    elif c in ("g", "f", "q"):
        # g: 10^5 x 4096 B at stride 4099 from an odd base; f: 10^5 x 3500 B
        # at stride 4128 from base 48 (one partial chunk per buffer, fixed
        # stride); q: 10^5 x 3500 B packed (stride 3500, some starts in a
        # page's first granule)
        n, L, S, off = {"g": (100_000, 4096, 4099, 3), "f": (100_000, 3500, 4128, 48),
                        "q": (100_000, 3500, 3500, 0)}[c]
        buf = torch.empty(off + n * S + 64, dtype=torch.uint8, device=dev)
        lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), buf.numel() // 8, 8, 0, 1, 0x5EED00B2, None)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        wsb = max(1, lib.nvl_crc32c_fixed_workspace_bytes(S, L, n))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        fn = lambda: lib.nvl_crc32c_fixed_dev(buf.data_ptr() + off, S, L, n, None, 0, out.data_ptr(), 0, ws.data_ptr(),
                                              wsb, st)
        alg = n * (L + 4)
        host = buf.cpu().numpy()
        check = lambda res: bool(np.array_equal(res, p.fixed(host[off:], S, L, n)))
    else:
        raise SystemExit(f"unknown config {c}")
    t = timeit(fn, a.reps if c != "4" else max(3, a.reps // 4))
    res = out.cpu().numpy().view(np.uint32)
    ps = SUSTAINED["period"]
    print(json.dumps({"config": c, "n": int(n), "bytes": int(alg), "median_us": round(t * 1e6, 1),
                      "GB/s": round(alg / t / 1e9, 1), "GiB/s": round(alg / t / 2**30, 1),
                      "frac_of_8TBs": round(alg / t / 8e12, 4), "sustained_period_us": round(ps * 1e6, 1),
                      "sustained_frac": round(alg / ps / 8e12, 4), "ok": bool(check(res))}), flush=True)
    del buf, keep
    torch.cuda.empty_cache()
