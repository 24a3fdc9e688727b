"""Interleaved A/B timing of kernel variants in ONE process (cdna guide §5.4 rule 24).

    python tools/ab_bench.py build/libnvl_crc32c_A.so build/libnvl_crc32c_B.so ...
Each .so is a full build of the C ABI; all run the config-2 fast path
(10^5 x 4 KiB) on the same device buffer, M rounds x R reps, HIP-event timed.
"""
import ctypes, os, sys, json, time
import numpy as np
import torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib

def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name); f.restype = res; f.argtypes = args
    return lib

def main():
    paths = sys.argv[1:]
    n = int(os.environ.get("AB_BLOCKS", "100000")); L = int(os.environ.get("AB_LEN", "4096"))
    rounds = int(os.environ.get("AB_ROUNDS", "12")); reps = int(os.environ.get("AB_REPS", "20"))
    dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
    libs = [load(p) for p in paths]
    for lib in libs:
        rc = lib.nvl_crc32c_init(0); assert rc == 0, (rc,)
    buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
    libs[0].nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
    outs = [torch.empty(n, dtype=torch.int32, device=dev) for _ in libs]
    ws = torch.empty(max([1] + [lib.nvl_crc32c_fixed_workspace_bytes(L, L, n) for lib in libs]), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    def run(k):
        rc = libs[k].nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, outs[k].data_ptr(), 0,
                                          ws.data_ptr(), ws.numel(), st)
        assert rc == 0
    times = [[] for _ in libs]
    walls = [[] for _ in libs]  # us per step of `reps` back-to-back launches, no events
    for k in range(len(libs)):
        for _ in range(3): run(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()  # ~100 ms of load first: the sustained-load state (the first ~30 ms run slower)
    while time.perf_counter() - t0 < 0.1:
        for k in range(len(libs)):
            for _ in range(5): run(k)
        torch.cuda.synchronize()
    periods = [[] for _ in libs]
    for r in range(rounds):
        ks = list(range(len(libs)))
        for k in ks[r % len(ks):] + ks[:r % len(ks)]:  # (rotated: no variant always follows the same one)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for j in range(reps):
                run(k)
            e1.record()
            torch.cuda.synchronize()
            periods[k].append(e0.elapsed_time(e1) * 1e3 / reps)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * reps)]
            for j in range(reps):
                ev[2*j].record(); run(k); ev[2*j+1].record()
            torch.cuda.synchronize()
            times[k] += [ev[2*j].elapsed_time(ev[2*j+1]) * 1e3 for j in range(reps)]
            t0 = time.perf_counter()
            for j in range(reps):
                run(k)
            torch.cuda.synchronize()
            walls[k].append((time.perf_counter() - t0) / reps * 1e6)
    ref = outs[0].cpu()
    for k, p in enumerate(paths):
        t = np.array(times[k]); same = bool(torch.equal(outs[k].cpu(), ref))
        gbs = n * (L + 4) / (np.median(t) * 1e-6) / 1e9
        print(json.dumps({"variant": os.path.basename(p), "median_us": round(float(np.median(t)), 2),
                          "min_us": round(float(t.min()), 2), "GB/s": round(gbs, 1), "frac": round(gbs / 8000, 4),
                          "wall_us_per_step": round(float(np.median(walls[k])), 2),
                          "period_us": round(float(np.median(periods[k])), 2),
                          "same_as_first": same}))

main()
