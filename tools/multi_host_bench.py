"""Host-resident batches through one GPU and through several pipes
(nvl_crc32c_batch_region_host vs nvl_crc32c_batch_region_host_multi), every
result checked against the engine's host CRC: the rate a caller with an
mmap'd table image sees (pageable memory in, CRCs out, synchronous).
    python tools/multi_host_bench.py [--devices 0,0] [--reps 5]
Shapes: `v` (10^5 x 4097 B at stride 4101, 410 MB: SSTable blocks | type) and
`big` (1 GiB: 256 x 4 MiB).  One JSON line per (shape, devices)."""
import argparse, json, os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from nvlevelz_amd import crc32c as C
from nvlevelz_amd import _lib

ap = argparse.ArgumentParser()
ap.add_argument("--devices", default="0|0,0|0,0,0,0")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
C.init(0)
rng = np.random.default_rng(1)
for shape in ("v", "big"):
    if shape == "v":
        n, L, S = 100_000, 4097, 4101
    else:
        n, L, S = 256, 4 << 20, 4 << 20
    img = rng.integers(0, 256, size=n * S, dtype=np.uint8)
    offs = (np.arange(n, dtype=np.uint64) * S)
    lens = np.full(n, L, dtype=np.uint64)
    want = None
    for dv in a.devices.split("|"):
        devs = [int(x) for x in dv.split(",")]
        run = (lambda: C.extend_region_host(img, offs, lens)) if len(devs) == 1 and devs == [0] else \
              (lambda: C.extend_region_host(img, offs, lens, devices=devs, min_bytes_per_device=1 << 20))
        got = run()
        if want is None:
            want = np.array([C.value(img[int(o):int(o) + L]) for o in offs[:2000]], dtype=np.uint32)
        ok = bool(np.array_equal(got[:2000], want))
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            run()
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        print(json.dumps({"shape": shape, "devices": devs, "bytes": int(n * L), "ms": round(t * 1e3, 2),
                          "GiB/s": round(n * L / t / 2**30, 2), "ok": ok,
                          "what": "pageable host image -> pinned staging -> H2D -> region kernel -> D2H, per pipe"}),
              flush=True)
