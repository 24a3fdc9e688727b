"""Where nvl_sstable_verify_table_dev's time goes on a 10^5-block table in
HBM: the whole call (wall, median), and the pieces it is made of timed alone
-- D2H of the records (24 B each) into pageable and pinned memory, a
host memcpy of the same bytes, one small D2H round trip, the CRC batch.
    python tools/diag/table_dev_time.py"""
import ctypes
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
nblocks, S = 100_000, 4096
image = bench.build_table_image(nblocks, S)
nbytes = len(image)
dimg = torch.frombuffer(bytearray(image), dtype=torch.uint8).to(dev)
cap = nblocks + 2
arr = (_lib.TableBlock * cap)()
n = ctypes.c_size_t(0)
st = ctypes.c_uint32(0)
nb = ctypes.c_uint64(0)
sptr = torch.cuda.current_stream().cuda_stream


def med(fn, reps=15):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(float(np.median(ts)) * 1e6, 1)


def call():
    assert L.nvl_sstable_verify_table_dev(dimg.data_ptr(), nbytes, arr, cap, ctypes.byref(n), ctypes.byref(st),
                                          ctypes.byref(nb), sptr) == 0


if os.environ.get("ONLY_CALL"):
    for _ in range(10):
        call()
    torch.cuda.synchronize()
    raise SystemExit(0)
rec = torch.empty(cap * 24, dtype=torch.uint8, device=dev)
pinned = torch.empty(cap * 24, dtype=torch.uint8, pin_memory=True)
page = np.zeros(cap * 24, dtype=np.uint8)
pg = torch.from_numpy(page)
small = torch.empty(64, dtype=torch.uint8, pin_memory=True)
out = {"call_us": med(call),
       "d2h_pageable_us": med(lambda: (pg.copy_(rec, non_blocking=False))),
       "d2h_pinned_us": med(lambda: (pinned.copy_(rec, non_blocking=True), torch.cuda.synchronize())),
       "host_memcpy_us": med(lambda: ctypes.memmove(arr, pinned.data_ptr(), cap * 24)),
       "small_roundtrip_us": med(lambda: (small.copy_(rec[:64], non_blocking=True), torch.cuda.synchronize()))}
print(out)
