"""Per-call latency of nvl_sstable_verify_table_dev against its floor: the
call (wall median) on tables of 63 .. 8181 blocks, beside one small D2H round
trip (pinned, hipMemcpyAsync + synchronize) and one region-kernel batch over
the same slots (hipEvent), so the host round trips the call makes can be
counted.     python tools/diag/table_dev_rt.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from nvlevelz_amd import _lib  # noqa: E402

L = _lib.lib
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
assert L.nvl_crc32c_init(0) == 0
sptr = torch.cuda.current_stream().cuda_stream


def med(fn, reps=41):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 1)


small = torch.empty(64, dtype=torch.uint8, pin_memory=True)
src = torch.empty(4096, dtype=torch.uint8, device=dev)
rt = med(lambda: (small.copy_(src[:64], non_blocking=True), torch.cuda.current_stream().synchronize()))
print(json.dumps({"small_d2h_roundtrip_us": rt}), flush=True)
for nblocks in [int(x) for x in os.environ.get("BLOCKS", "63,511,2045,8181").split(",")]:
    image = bench.build_table_image(nblocks, 4096)
    nbytes = len(image)
    dimg = torch.frombuffer(bytearray(image), dtype=torch.uint8).to(dev)
    cap = nblocks + 8
    arr = (_lib.TableBlock * cap)()
    n, st, nb = ctypes.c_size_t(0), ctypes.c_uint32(0), ctypes.c_uint64(0)

    def call():
        rc = L.nvl_sstable_verify_table_dev(dimg.data_ptr(), nbytes, arr, cap, ctypes.byref(n), ctypes.byref(st),
                                            ctypes.byref(nb), sptr)
        assert rc == 0 and st.value == 0 and nb.value == 0, (rc, st.value, nb.value)

    print(json.dumps({"blocks": nblocks, "table_bytes": nbytes, "call_us": med(call), "n_blocks": n.value}),
          flush=True)
