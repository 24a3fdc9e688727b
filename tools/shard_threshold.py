"""When does spreading a device-resident batch of n 4 KiB blocks over G GPUs
pay (VERDICT r05 missing #1)?  The pieces measured on ONE MI355X, the rest a
stated model -- this pool lends no multi-GPU node:

  t_call(n)     one nvl_crc32c_fixed_dev call from an idle queue (event pair,
                synchronize after each; median) -- a shard's kernel
  t_enq         the host time to enqueue one such call (the single-process
                multi-device entry, nvl_crc32c_fixed_dev_multi, enqueues its
                shards one after another)
  t_gather(n,G) nvl_crc32c_gather_dev of G shards' results in config 5's
                round-robin order with every shard on this device (device
                copies + the interleave kernel: the gather without the link)
  link          (G-1)/G * 4n bytes over xGMI at LINK_GBPS per peer copy (153
                GB/s per link, the copies one after another on the
                destination's stream: no overlap assumed)

  one process per GPU (bench.py --gpus G):  T = t_call(n/G)
       + when rank 0 needs every CRC: t_gather(n, G) + link
  one process, G devices (fixed_dev_multi): T = (G-1) t_enq + t_call(n/G)
       (+ the same gather)
  sharding pays where T < t_call(n).
    python tools/shard_threshold.py [--out profiles/r06/shard_threshold.json]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path.insert(0, ROOT)
from nvlevelz_amd import _lib  # noqa: E402

LINK_GBPS = 153.0
ap = argparse.ArgumentParser()
ap.add_argument("--out", default=None)
a = ap.parse_args()
L = _lib.lib
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
assert L.nvl_crc32c_init(0) == 0
st = torch.cuda.current_stream().cuda_stream
NMAX = 10_000_000
buf = torch.empty(NMAX * 4096, dtype=torch.uint8, device=dev)
assert L.nvl_crc32c_fill_splitmix(buf.data_ptr(), NMAX, 4096, 0, 1, 0x5EED0005, None) == 0
out = torch.empty(NMAX, dtype=torch.int32, device=dev)


def call(n):
    rc = L.nvl_crc32c_fixed_dev(buf.data_ptr(), 4096, 4096, n, None, 0, out.data_ptr(), 0, None, 0, st)
    assert rc == 0, rc


def t_call(n, reps=25):
    for _ in range(5):
        call(n)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call(n)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


def t_enq(n=100_000, reps=50):
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        call(n)
        ts.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    return float(np.median(ts))


def t_gather(n, G, reps=15):
    per = [(n - k + G - 1) // G for k in range(G)]
    shards = (_lib.Shard * G)()
    pos = 0
    for k in range(G):
        shards[k].device = 0
        shards[k].base = None
        shards[k].stride = 4096
        shards[k].len = 4096
        shards[k].n = per[k]
        shards[k].out = out.data_ptr() + 4 * pos
        shards[k].stream = None
        pos += per[k]
    dst = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    g = lambda: L.nvl_crc32c_gather_dev(dst.data_ptr(), 0, shards, G, _lib.GATHER_ROUND_ROBIN, None)
    for _ in range(3):
        assert g() == 0
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.default_stream())
        assert g() == 0
        e1.record(torch.cuda.default_stream())
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return float(np.median(ts))


sizes = [1_000, 3_000, 10_000, 30_000, 100_000, 300_000, 1_000_000, 3_000_000, 10_000_000]
calls = {}
for n in sorted(set(sizes + [max(1, s // G) for s in sizes for G in (2, 4, 8)])):
    calls[n] = t_call(n)
enq = t_enq()
rows = []
for n in sizes:
    row = {"n": n, "bytes": n * 4096, "t_call_us": round(calls[n], 2)}
    for G in (2, 4, 8):
        k = calls[max(1, n // G)]
        gat = t_gather(n, G)
        link = (G - 1) / G * 4 * n / (LINK_GBPS * 1e3)  # us
        row[f"G{G}"] = {"t_shard_us": round(k, 2), "gather_us": round(gat, 2), "link_us": round(link, 2),
                        "multi_process_us": round(k, 2), "multi_process_gathered_us": round(k + gat + link, 2),
                        "one_process_us": round((G - 1) * enq + k, 2),
                        "speedup_multi_process": round(calls[n] / k, 2),
                        "speedup_one_process_gathered": round(calls[n] / ((G - 1) * enq + k + gat + link), 2)}
    rows.append(row)
    print(json.dumps(row), flush=True)
res = {"what": __doc__.split("\n\n")[0], "t_enqueue_us": round(enq, 2), "link_GBps_assumed": LINK_GBPS, "rows": rows}
for G in (2, 4, 8):
    for key in ("speedup_multi_process", "speedup_one_process_gathered"):
        first = next((r["n"] for r in rows if r[f"G{G}"][key] > 1.0), None)
        res[f"pays_from_n_G{G}_{key[8:]}"] = first
print(json.dumps({k: v for k, v in res.items() if k != "rows"}), flush=True)
if a.out:
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
