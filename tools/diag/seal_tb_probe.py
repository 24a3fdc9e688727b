"""Where the forced-GPU seal inside the reference TableBuilder build spends
its time (DESIGN §9 anomaly): builds the same ~1.8 MB table R times with the
host seal and with the GPU seal through shims::BatchingWritableFile, and times
nvl_sstable_seal_trailers alone on the built image.  Run under
`rocprofv3 --hip-runtime-trace --stats` to see the HIP calls per build.
    python tools/diag/seal_tb_probe.py [R]"""
import ctypes, json, os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
import torch  # noqa: F401
from nvlevelz_amd import _lib
import oracle
L = _lib.lib
assert L.nvl_crc32c_init(0) == 0
R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
rt = oracle.ref_table(deferred=True)
rng = np.random.default_rng(5)
nk = int(2**21 / 120)
keys = [b"key%013d" % i for i in range(nk)]
vals = [rng.integers(0, 256, 100, dtype=np.uint8).tobytes() for _ in range(nk)]
for eng, fl in (("host", _lib.FRAMING_HOST), ("gpu", _lib.FRAMING_GPU), ("host", _lib.FRAMING_HOST),
                ("gpu", _lib.FRAMING_GPU)):
    ts = []
    for _ in range(R):
        t0 = time.perf_counter()
        img, _ = rt.build(keys, vals, via_shim=1, seal_flags=fl)
        ts.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"build_with_seal": eng, "ms": [round(t, 2) for t in ts], "seals": rt.seals}), flush=True)
