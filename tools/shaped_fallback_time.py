"""Cost of NVL_CRC32C_FLAG_REGION_SHAPED on batches that are NOT region-shaped
(the region kernel's per-buffer path; nvl_sstable_verify_table_dev passes the
flag for every table, so this is what a corrupt / crafted out-of-order index
costs): per call against the routed (checked) entry on the same batch.
    python tools/shaped_fallback_time.py"""
import json, os, sys, time
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from nvlevelz_amd import crc32c as C

C.init(0)
dev = torch.device("cuda:0")
rng = np.random.default_rng(4)
for name, n in (("r_shuffled_1e4", 10_000), ("r_shuffled_1e5", 100_000), ("r_sorted_1e5", 100_000)):
    lens = rng.integers(3364, 4110, n)
    offs = np.cumsum(lens + 4) - lens - 4
    img = torch.empty(int(offs[-1] + lens[-1]) + 64, dtype=torch.uint8, device=dev)
    C.fill_splitmix(img, img.numel() // 8, 8, 0x77)
    perm = rng.permutation(n) if "shuffled" in name else np.arange(n)
    to = torch.from_numpy(offs[perm].astype(np.int64)).to(dev)
    tl = torch.from_numpy(lens[perm].astype(np.int64)).to(dev)
    res = {"batch": name}
    ref = None
    for shaped in (False, True):
        out = C.extend_region(img, to, tl, shaped=shaped)
        torch.cuda.synchronize()
        got = C.to_u32(out)
        ref = got if ref is None else ref
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            C.extend_region(img, to, tl, shaped=shaped)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res["shaped_ms" if shaped else "checked_ms"] = round(float(np.median(ts)) * 1e3, 3)
        res["same"] = bool(np.array_equal(got, ref))
    print(json.dumps(res), flush=True)
