"""Host-resident batches through one GPU and through several pipes
(nvl_crc32c_batch_region_host vs nvl_crc32c_batch_region_host_multi), every
result checked against the engine's host CRC: the rate a caller with an
mmap'd table image sees (host memory in, CRCs out, synchronous).
    python tools/multi_host_bench.py [--devices 0|0,0|0,0,0,0] [--reps 5] [--modes staged,dma,zero]
Shapes: `v` (10^5 x 4097 B at stride 4101, 410 MB: SSTable blocks | type) and
`big` (1 GiB: 256 x 4 MiB).  Modes:
  staged -- pageable image -> pinned staging (CPU copy, 1-4 threads) -> H2D
  dma    -- image registered once (nvl_crc32c_host_register): H2D DMA straight
            from its pages, no CPU copy
  zero   -- registered, NVL_CRC32C_FLAG_HOST_ZERO_COPY: the kernels read the
            pages in place over PCIe (no H2D copy at all)
One JSON line per (shape, mode, devices): wall GiB/s (median of reps) and the
process's host CPU-seconds per GiB checksummed (getrusage user + sys over
every thread, around the timed reps) -- what the call costs the host cores,
beside the reference CPU leg's 1 / per-core rate."""
import argparse, json, os, resource, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvlevelz_amd import crc32c as C


def cpu_s():
    r = resource.getrusage(resource.RUSAGE_SELF)
    return r.ru_utime + r.ru_stime


ap = argparse.ArgumentParser()
ap.add_argument("--devices", default="0|0,0|0,0,0,0")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--modes", default="staged,dma,zero")
ap.add_argument("--shapes", default="v,big")
a = ap.parse_args()
C.init(0)
rng = np.random.default_rng(1)
for shape in a.shapes.split(","):
    if shape == "v":
        n, L, S = 100_000, 4097, 4101
    else:
        n, L, S = 256, 4 << 20, 4 << 20
    img = rng.integers(0, 256, size=n * S, dtype=np.uint8)
    offs = (np.arange(n, dtype=np.uint64) * S)
    lens = np.full(n, L, dtype=np.uint64)
    want = np.array([C.value(img[int(o):int(o) + L]) for o in offs[:2000]], dtype=np.uint32)
    for mode in a.modes.split(","):
        reg_ms = None
        if mode in ("dma", "zero"):
            t0 = time.perf_counter()
            C.host_register(img)
            reg_ms = (time.perf_counter() - t0) * 1e3
        try:
            for dv in a.devices.split("|"):
                devs = [int(x) for x in dv.split(",")]
                zc = mode == "zero"
                run = (lambda: C.extend_region_host(img, offs, lens, zero_copy=zc)) if devs == [0] else \
                      (lambda: C.extend_region_host(img, offs, lens, devices=devs, min_bytes_per_device=1 << 20,
                                                    zero_copy=zc))
                got = run()
                ok = bool(np.array_equal(got[:2000], want))
                ts = []
                c0 = cpu_s()
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    got = run()
                    ts.append(time.perf_counter() - t0)
                c1 = cpu_s()
                ok = ok and bool(np.array_equal(got[:2000], want))
                t = float(np.median(ts))
                gib = n * L / 2**30
                print(json.dumps({"shape": shape, "mode": mode, "devices": devs, "bytes": int(n * L),
                                  "ms": round(t * 1e3, 2), "GiB/s": round(n * L / t / 2**30, 2), "ok": ok,
                                  "host_cpu_s_per_GiB": round((c1 - c0) / (a.reps * gib), 4),
                                  "register_ms": None if reg_ms is None else round(reg_ms, 1),
                                  "what": {"staged": "pageable image -> pinned staging -> H2D -> kernel -> D2H",
                                           "dma": "registered image -> H2D DMA from its pages -> kernel -> D2H",
                                           "zero": "registered image read in place by the kernel over PCIe -> D2H"}
                                  [mode] + ", per pipe"}), flush=True)
        finally:
            if mode in ("dma", "zero"):
                C.host_unregister(img)
