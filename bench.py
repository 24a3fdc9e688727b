#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC32C over 4 KiB blocks on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A "step" = one pass of the hot path (nvl_crc32c_fixed_dev through the C ABI)
over one batch of synthetic, already-HBM-resident 4 KiB blocks.

Workloads (BASELINE.json configs):
  cfg2 (default): 10^5 x 4 KiB blocks PER GPU (weak scaling).  Rank r holds
        global blocks r, r+N, r+2N, ... (round-robin shard, generated in place
        from the canonical splitmix64 stream).  At N=1 this is
        exactly BASELINE config 2.
  cfg5: 10^7 x 4 KiB blocks in total, round-robin over the N GPUs (strong).

No data-path collective: every block's CRC is independent, so shards never
exchange bytes; only the timing max and a verification digest cross ranks
(outside the timed region).

The JSON line adds
  roofline     -- dominant kernel: algorithmic bytes per launch (4096+4 B per
                  block) / its mean duration from HIP events recorded on the
                  launch stream, against the 8 TB/s HBM3E peak.  `traffic` is
                  the PMC-measured HBM bytes per launch from
                  profiles/pmc_traffic.json when present (rocprofv3, corrected
                  per MI355X_MICROARCH.md §HBM), else null.
  cpu_baseline -- the reference's own util/crc32c.cc + port/port_posix_sse.cc
                  (oracle/_ref, kind "reference"; the clean-room port, kind
                  "port", if _ref is absent) timed on this host's cores on a
                  bounded sample of the same blocks (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s device-resident batched CRC32C over 4 KiB blocks; % HBM-read roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BLOCK = 4096
SEED_CFG2 = 0x5EED0001
SEED_CFG5 = 0x5EED0005


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", choices=["cfg2", "cfg5"], default="cfg2")
    ap.add_argument("--blocks", type=int, default=None, help="override blocks per GPU (cfg2)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="target seconds per CPU-baseline leg (all-core and 1-thread)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--e2e", action="store_true", help="also time host->device->host end to end")
    ap.add_argument("--shims", action="store_true",
                    help="also time the whole-table verify shim on a host-resident 10^5-block SSTable image")
    ap.add_argument("--verify", action="store_true", default=True)
    return ap.parse_args()


def cpu_baseline(host: np.ndarray, n: int, seconds: float, threads: int) -> dict:
    import oracle
    kind = "reference" if oracle.ref_available("sse") else "port"
    impl = oracle.ref("sse") if kind == "reference" else oracle.port()

    def run(nblk, th):
        if kind == "reference":
            return impl.fixed_mt(host, BLOCK, BLOCK, nblk, th)
        return impl.fixed_mt(host, BLOCK, BLOCK, nblk, th, False)

    def timed(nblk, th):
        run(min(nblk, 2000), th)  # warm
        reps, t0 = 0, time.perf_counter()
        while True:
            r = run(nblk, th)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return r, reps * nblk * BLOCK / el / 2**30, reps, el

    th = max(1, min(threads, os.cpu_count() or 1))
    r_all, gibs_all, reps_all, el_all = timed(n, th)
    r_one, gibs_one, reps_one, el_one = timed(min(n, 20000), 1)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {
        "value": round(gibs_all, 3), "unit": "GiB/s", "cores": th, "kind": kind,
        "sample": f"{reps_all} passes over the first {n} x 4 KiB blocks of this rank's batch "
                  f"({el_all:.1f} s, {th} threads, contiguous partition), "
                  f"leveldb::crc32c::Value via port::AcceleratedCRC32C (SSE4.2)",
        "single_thread": {"value": round(gibs_one, 3), "unit": "GiB/s", "cores": 1,
                          "sample": f"{reps_one} passes over {min(n, 20000)} blocks ({el_one:.1f} s)"},
        "host_cpu": model, "host_nproc": os.cpu_count(),
        "_check": r_all,
    }


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def shim_bench(nblocks: int = 100_000) -> dict:
    """nvl_sstable_verify_table (include/nvl_framing.h) over a host-resident
    SSTable image of `nblocks` 4 KiB data blocks (table/format.h layout: one
    key-value entry + restart array per block, 5-byte trailers, an index with
    one BlockHandle per block, an empty metaindex, the 48-byte footer), as a
    caller with an mmap'd table would run it: file bytes in host memory ->
    one staging copy + H2D + batch kernel + D2H of the CRCs.  Beside it, the
    same walk with the host CRC (NVL_FRAMING_HOST) and, where the reference
    build exists, the reference's own Footer/ReadBlock/Block::Iter scan
    (oracle/_ref, single thread) -- the CPU legs are reported baselines."""
    import ctypes
    from nvlevelz_amd import _lib
    L = _lib.lib
    S = 4096
    key_len = 16
    hdr = _varint(0) + _varint(key_len)
    vlen = S - 8 - key_len - len(hdr) - 2
    hdr += _varint(vlen)
    assert len(hdr) + key_len + vlen + 8 == S
    stride = S + 5
    rng = np.random.default_rng(2024)
    img = np.zeros((nblocks, stride), dtype=np.uint8)
    img[:, :len(hdr)] = np.frombuffer(hdr, dtype=np.uint8)
    keys = np.frombuffer(b"".join(b"k%015d" % i for i in range(nblocks)), dtype=np.uint8).reshape(nblocks, key_len)
    img[:, len(hdr):len(hdr) + key_len] = keys
    img[:, len(hdr) + key_len:S - 8] = rng.integers(0, 256, size=(nblocks, vlen), dtype=np.uint8)
    img[:, S - 4] = 1  # num_restarts = 1, restart[0] = 0
    data = bytearray(img.reshape(-1).tobytes())
    del img
    handles = np.stack([np.arange(nblocks, dtype=np.uint64) * stride, np.full(nblocks, S, np.uint64)], 1)
    cbuf = (ctypes.c_char * len(data)).from_buffer(data)
    rc = L.nvl_sstable_seal_trailers(cbuf, len(data), np.ascontiguousarray(handles).ctypes.data, nblocks, 0)
    del cbuf
    assert rc == 0, rc

    def raw_block(contents: bytes) -> tuple:
        off = len(data)
        data.extend(contents + b"\0" + bytes(4))
        h = np.array([[off, len(contents)]], dtype=np.uint64)
        cb = (ctypes.c_char * len(data)).from_buffer(data)
        assert L.nvl_sstable_seal_trailers(cb, len(data), h.ctypes.data, 1, _lib.FRAMING_HOST) == 0
        del cb
        return off, len(contents)

    meta_h = raw_block((0).to_bytes(4, "little") + (1).to_bytes(4, "little"))
    parts, restarts, pos = [], [], 0
    for i in range(nblocks):  # index block, restart interval 1 (table_builder.cc)
        v = _varint(i * stride) + _varint(S)
        e = _varint(0) + _varint(key_len) + _varint(len(v)) + (b"k%015d" % i) + v
        restarts.append(pos)
        pos += len(e)
        parts.append(e)
    index = b"".join(parts) + np.array(restarts, dtype="<u4").tobytes() + len(restarts).to_bytes(4, "little")
    index_h = raw_block(index)
    foot = _varint(meta_h[0]) + _varint(meta_h[1]) + _varint(index_h[0]) + _varint(index_h[1])
    data.extend(foot + bytes(40 - len(foot)) + (0xDB4775248B80FB57).to_bytes(8, "little"))
    image = bytes(data)
    del data
    nbytes = len(image)

    cap = nblocks + 2
    arr = (_lib.TableBlock * cap)()
    n = ctypes.c_size_t(0)
    st = ctypes.c_uint32(0)
    nb = ctypes.c_uint64(0)

    def run(flags):
        rc = L.nvl_sstable_verify_table(image, nbytes, arr, cap, ctypes.byref(n), ctypes.byref(st), ctypes.byref(nb),
                                        flags)
        assert rc == 0 and st.value == 0 and n.value == cap and nb.value == 0, (rc, st.value, n.value, nb.value)

    def timed(fn, reps):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    t_gpu = timed(lambda: run(0), 7)
    t_host = timed(lambda: run(_lib.FRAMING_HOST), 3)
    res = {"what": "nvl_sstable_verify_table on a host-resident table image (footer -> index -> every block), "
                   "wall clock per call, median",
           "table": {"data_blocks": nblocks, "block_bytes": S, "file_bytes": nbytes},
           "gpu": {"ms": round(t_gpu * 1e3, 3), "GiB/s": round(nbytes / t_gpu / 2**30, 3),
                   "path": "host image -> pinned staging -> H2D -> one batch kernel -> D2H"},
           "host_crc": {"ms": round(t_host * 1e3, 3), "GiB/s": round(nbytes / t_host / 2**30, 3), "cores": 1,
                        "path": "same walk, NVL_FRAMING_HOST"}}
    try:
        import oracle
        if oracle.ref_framing_available():
            rf = oracle.ref_framing()
            need = len(rf.table_scan(image)) + 1  # sizes the trace buffer once
            tr = []
            t_ref = timed(lambda: tr.append(rf.table_scan(image, need)), 3)
            ok = tr[-1].count(" OK\n") == cap
            res["cpu_reference"] = {"ms": round(t_ref * 1e3, 3), "GiB/s": round(nbytes / t_ref / 2**30, 3),
                                    "cores": 1, "all_blocks_ok": ok,
                                    "path": "reference Footer::DecodeFrom + ReadBlock(verify_checksums) + "
                                            "Block::Iter over index and metaindex (oracle/_ref, SSE4.2 crc32c)"}
    except Exception as e:  # the CPU leg is a reported baseline only
        res["cpu_reference"] = {"error": repr(e)}
    return res


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from nvlevelz_amd import crc32c

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"[bench] --gpus {args.gpus} needs torch.distributed.run; running 1 rank", file=sys.stderr)
        args.gpus = world
    # NVL_BENCH_BACKEND=gloo rehearses the N-rank path on fewer GPUs (ranks
    # share devices round-robin); the default is RCCL with one GPU per rank.
    backend = os.environ.get("NVL_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", local % ndev if backend == "gloo" else local)
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)  # RCCL; timing/verification only
    red_dev = torch.device("cpu") if backend == "gloo" else dev
    crc32c.init(dev.index)

    N = world
    if args.config == "cfg2":
        n_local = args.blocks or 100_000
        seed = SEED_CFG2
        workload = (f"cfg2: {n_local} x 4 KiB blocks per GPU (BASELINE config 2 at N=1), device-resident, "
                    f"stride 4096, round-robin global block ids rank+k*N")
        scaling = "weak"
    else:
        total = 10_000_000
        n_local = (total - rank + N - 1) // N
        seed = SEED_CFG5
        workload = f"cfg5: 10^7 x 4 KiB blocks total, round-robin over {N} GPU(s)"
        scaling = "strong"

    buf = torch.empty(n_local * BLOCK, dtype=torch.uint8, device=dev)
    crc32c.fill_splitmix(buf, n_local, BLOCK, seed, first_block=rank, block_step=N)
    stream = torch.cuda.current_stream(dev)
    batch = crc32c.FixedBatch(buf, BLOCK, BLOCK, n_local, stream=stream)  # validated once
    out = batch.out
    step = batch.launch  # one C call per step; the host stays ahead of the GPU

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # --- verification (untimed) --------------------------------------------
    verify = {}
    res = crc32c.to_u32(out)
    if rank == 0:
        if args.config == "cfg2":
            verify["crc0"] = hex(int(res[0]))
            verify["crc0_ok"] = int(res[0]) == 0x6104AC89
            if N == 1 and n_local == 100_000:
                # digest = Value() of the little-endian CRC array, golden from the reference
                with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
                    g = json.load(f)["cfg2"]
                d = crc32c.value(np.ascontiguousarray(res, dtype="<u4").tobytes())
                verify["digest"] = hex(d)
                verify["digest_ok"] = d == g["digest"]
        else:  # cfg5: block 0 of rank 0 is global block 0; cross-check with the host CRC
            h0 = crc32c.value(buf[:BLOCK].cpu().numpy().tobytes())
            verify["crc0"] = hex(int(res[0]))
            verify["crc0_matches_host"] = int(res[0]) == h0

    # --- timed region ------------------------------------------------------
    # K back-to-back launches, nothing else enqueued between them (an event per
    # launch would add a marker packet to every step).  Two HIP events on the
    # launch stream bracket the region: their interval / K is the mean launch
    # duration used for the roofline -- it includes the inter-launch gaps, so
    # it is conservative against rocprofv3's per-kernel durations.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    region_ms = ev0.elapsed_time(ev1)
    # Untimed: per-launch kernel durations (events bracketing each launch), the
    # quantity rocprofv3's kernel trace reports, for cross-checking.
    kev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * min(args.steps, 100))]
    for k in range(len(kev) // 2):
        kev[2 * k].record(stream)
        step()
        kev[2 * k + 1].record(stream)
    torch.cuda.synchronize()
    kern_ms = [kev[2 * k].elapsed_time(kev[2 * k + 1]) for k in range(len(kev) // 2)]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        nt = torch.tensor([n_local], dtype=torch.int64, device=red_dev)
        dist.all_reduce(nt, op=dist.ReduceOp.SUM)
        total_blocks = int(nt.item())
    else:
        total_blocks = n_local

    value = total_blocks * BLOCK * args.steps / elapsed / 2**30
    mean_kern_s = region_ms / args.steps / 1e3
    med_kern_s = float(np.median(kern_ms)) / 1e3
    alg_bytes = n_local * (BLOCK + 4)  # every input byte once + 4 B CRC out
    achieved = alg_bytes / mean_kern_s / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pj = json.load(f)
            if pj.get("blocks") == n_local:
                traffic = pj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    cpu = None
    e2e = None
    if rank == 0 and N == 1 and not args.no_cpu:
        host = buf.cpu().numpy()
        cpu = cpu_baseline(host, n_local, args.cpu_seconds, args.cpu_threads)
        chk = cpu.pop("_check")
        verify["cpu_matches_gpu"] = bool(np.array_equal(chk, res[:chk.size]))
    if rank == 0 and args.e2e:
        pinned = torch.empty(n_local * BLOCK, dtype=torch.uint8).pin_memory()
        pinned.copy_(buf.cpu())
        hp = pinned.numpy()
        crc32c.extend_fixed_host(hp, BLOCK, BLOCK, n_local)
        t1 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            r = crc32c.extend_fixed_host(hp, BLOCK, BLOCK, n_local)
        el = time.perf_counter() - t1
        e2e = {"value": round(n_local * BLOCK * reps / el / 2**30, 3), "unit": "GiB/s",
               "what": "pinned host -> H2D -> kernel -> D2H of u32 results, 2-stream pipelined, synchronous",
               "ok": bool(np.array_equal(r, res))}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": N,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 stream, SURVEY.md §8d), generated in HBM",
            "config": {"workload": workload, "blocks_per_gpu": n_local, "block_bytes": BLOCK,
                       "parallelism": f"{N} independent shard(s), no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "crc32c_fixed_kernel<0> (aligned 4 KiB blocks, scheduler A)",
                         "alg_bytes_per_launch": alg_bytes,
                         "mean_launch_us": round(mean_kern_s * 1e6, 2),
                         "mean_launch_what": "HIP events bracketing the K timed launches / K (incl. inter-launch gaps)",
                         "median_kernel_us": round(med_kern_s * 1e6, 2),
                         "median_kernel_what": "untimed pass, events around each launch (rocprofv3-comparable)"},
            "cpu_baseline": cpu,
            "verify": verify,
        }
        if e2e:
            line["e2e"] = e2e
        if args.shims and N == 1:
            line["shims"] = shim_bench()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
