#!/usr/bin/env python3
"""bench.py -- device-resident batched CRC32C over 4 KiB blocks on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config cfg2|cfg5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Without a torch.distributed launcher (no WORLD_SIZE in the environment),
`--gpus N` > 1 makes this process start the N ranks itself (one child process
per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) before anything touches a
GPU; the parent only waits for them (rank 0 prints the line).

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
                  block) / its average launch duration in the timed region
                  (HIP events on the launch stream around the K launches / K),
                  against the 8 TB/s HBM3E peak.  `traffic` is the committed
                  PMC-measured HBM bytes per launch (profiles/pmc_traffic.json,
                  rocprofv3 --pmc passes: L2 memory-side request counts by
                  size, MI355X_MICROARCH.md §HBM), labelled as such, else null.
  cfg5         -- BASELINE config 5 on the same N ranks (every run, N = 1
                  included): 10^7 x 4 KiB blocks in total round-robin over
                  the N GPUs (strong scaling), its GiB/s, frac, and every
                  rank's digest verified (cfg5_leg).  The headline `value`
                  stays config 2 (weak scaling: N = 1 is BASELINE config 2).
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
    ap.add_argument("--warmup", type=int, default=1000)  # ~67 ms: past the ~30 ms ramp of a sustained load (profiles/r04_clocks_cfg2.jsonl)
    ap.add_argument("--config", choices=["cfg2", "cfg5"], default="cfg2")
    ap.add_argument("--blocks", type=int, default=None, help="override blocks per GPU (cfg2)")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="target seconds per CPU-baseline leg (all-core and 1-thread)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the all-core CPU leg (0 = the physical cores this process may run on, capped by its cgroup CPU quota)")
    ap.add_argument("--cfg5-steps", type=int, default=20,
                    help="timed steps of the BASELINE config-5 leg (10^7 blocks in total, round-robin over the N "
                         "GPUs, strong scaling) reported beside the headline; 0 = skip")
    ap.add_argument("--cfg5-warmup", type=int, default=5)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host->device->host end-to-end leg (N=1)")
    ap.add_argument("--shims", action="store_true",
                    help="also time the whole-table verify shim on a host-resident 10^5-block SSTable image")
    ap.add_argument("--verify", action="store_true", default=True)
    ap.add_argument("--probe", type=int, default=200,
                    help="launches of the read-only probe kernel timed after the timed region (0: skip)")
    ap.add_argument("--sustained", type=int, default=2000,
                    help="untimed back-to-back launches after the timed region (segment periods; 0 = skip)")
    return ap.parse_args()


def physical_cores() -> tuple:
    """(physical cores, logical CPUs) among the CPUs this process may run on:
    SMT siblings (thread_siblings_list) count once."""
    cpus = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                cores.add(f.read().strip())
        except OSError:
            cores.add(str(c))
    return len(cores), len(cpus)


def cgroup_cpu_max() -> str | None:
    """The cgroup v2 CPU quota of this process ("max 100000" = none)."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = f.read().strip().split("\n")[0].split("::", 1)[-1]
        for path in (f"/sys/fs/cgroup{rel}/cpu.max", "/sys/fs/cgroup/cpu.max"):
            if os.path.exists(path):
                with open(path) as f:
                    return f.read().strip()
    except OSError:
        pass
    return None


def cgroup_cpus() -> int | None:
    """CPUs the cgroup v2 quota allows this process (ceil(quota / period)), None without a quota."""
    cm = cgroup_cpu_max()
    try:
        q, per = cm.split()
        return None if q == "max" else max(1, -(-int(q) // int(per)))
    except (AttributeError, ValueError):
        return None


def cpu_baseline(host: np.ndarray, n: int, seconds: float, threads: int, reps: int = 5) -> dict:
    """The reference's own util/crc32c.cc + port/port_posix_sse.cc (oracle/_ref;
    the clean-room port if absent) on this host: one thread per physical core
    the process may use (capped by the cgroup CPU quota; the uncapped
    all-physical-core figure beside it), and one thread.  Each leg is `reps` timed repetitions (median reported);
    one repetition = `passes` passes over each thread's contiguous share of the
    first n blocks inside ONE call (thread start-up paid once), sized from a
    calibration call to ~seconds/reps.  Around every repetition the process's
    CPU seconds (os.times, all threads) are read: CPU-seconds / wall = the
    parallelism that actually ran, reported as `cores` -- a cgroup quota or a
    busy host shows there, not in the thread count.  Plus the drop-in's own
    single-buffer path (`single_buffer`): db/db_bench.cc:729-746's crc32c loop
    (Value() of one 4 KiB buffer until 500 MB) through the reference's Value
    and through nvl_crc32c_value on one core."""
    import oracle
    kind = "reference" if oracle.ref_available("sse") else "port"
    impl = oracle.ref("sse") if kind == "reference" else oracle.port()

    def run(nblk, th, passes):
        return impl.fixed_mt(host, BLOCK, BLOCK, nblk, th, reps=passes)

    def leg(nblk, th):
        t0 = time.perf_counter()
        r = run(nblk, th, 1)  # calibration (also warms the pages)
        one = max(time.perf_counter() - t0, 1e-4)
        passes = max(1, int(seconds / reps / one))
        rates, par = [], []
        for _ in range(reps):
            c0, t0 = os.times(), time.perf_counter()
            run(nblk, th, passes)
            el = time.perf_counter() - t0
            c1 = os.times()
            rates.append(passes * nblk * BLOCK / el / 2**30)
            par.append(((c1.user - c0.user) + (c1.system - c0.system)) / el)
        return r, float(np.median(rates)), float(np.median(par)), passes, rates

    phys, logical = physical_cores()
    quota = cgroup_cpus()
    # one thread per CPU the process may actually use: the physical cores of
    # its affinity set, capped by the cgroup quota (more threads than the
    # quota only time-slice; that figure is reported beside it)
    th = threads if threads > 0 else min(phys, quota or phys)
    r_all, gibs_all, par_all, passes_all, rates_all = leg(n, th)
    over = None
    if threads <= 0 and phys > th:
        _, g_o, p_o, pa_o, r_o = leg(n, phys)
        over = {"value": round(g_o, 3), "unit": "GiB/s", "threads": phys, "effective_parallelism": round(p_o, 2),
                "repetitions_gibs": [round(x, 2) for x in r_o],
                "what": "the same leg on one thread per physical core of the affinity set, above the cgroup quota"}
    n1 = min(n, 20000)
    _, gibs_one, par_one, passes_one, rates_one = leg(n1, 1)
    single = None
    if kind == "reference" and hasattr(impl.lib, "ref_dbbench_crc32c"):
        import ctypes
        from nvlevelz_amd import _lib
        fn = ctypes.cast(_lib.lib.nvl_crc32c_value, ctypes.c_void_p).value
        ref_r, nvl_r = [], []
        for _ in range(reps):
            g, c_ref = impl.dbbench_crc32c(None)
            ref_r.append(g)
            g, c_nvl = impl.dbbench_crc32c(fn)
            nvl_r.append(g)
        single = {"reference": round(float(np.median(ref_r)), 3), "nvl_crc32c_value": round(float(np.median(nvl_r)), 3),
                  "unit": "GiB/s", "cores": 1, "ratio": round(float(np.median(nvl_r) / np.median(ref_r)), 3),
                  "same_crc": c_ref == c_nvl,
                  "what": "db/db_bench.cc:729-746 crc32c loop: Value() of one 4 KiB buffer until 500 MB, one "
                          "thread; the reference's leveldb::crc32c::Value (oracle/_ref, SSE4.2 crc32q) against "
                          "the drop-in's nvl_crc32c_value (include/nvl_crc32c.h; integration/"
                          "leveldb_util_crc32c.cc forwards Extend to it), median of 5 alternating runs"}
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
        "value": round(gibs_all, 3), "unit": "GiB/s", "cores": int(round(par_all)), "kind": kind,
        "threads": th, "effective_parallelism": round(par_all, 2),
        "per_thread_gibs": round(gibs_all / max(par_all, 1e-9), 3),
        "cpu_s_per_GiB": round(par_all / gibs_all, 4),
        "sample": f"median of {reps} repetitions x {passes_all} passes over the first {n} x 4 KiB blocks of this "
                  f"rank's batch ({th} threads = the physical cores of the {logical} CPUs in this process's "
                  f"affinity set ({phys}) capped by the cgroup quota ({quota} CPUs), contiguous share per thread; "
                  f"cores = CPU-seconds / wall of the run = {par_all:.1f}), leveldb::crc32c::Value via "
                  f"port::AcceleratedCRC32C (SSE4.2)",
        "repetitions_gibs": [round(x, 2) for x in rates_all],
        "cgroup_cpu_max": cgroup_cpu_max(), "cgroup_cpus": quota,
        "threads_over_quota": over,
        "single_thread": {"value": round(gibs_one, 3), "unit": "GiB/s", "cores": 1,
                          "effective_parallelism": round(par_one, 2),
                          "sample": f"median of {reps} x {passes_one} passes over {n1} blocks",
                          "repetitions_gibs": [round(x, 2) for x in rates_one]},
        "single_buffer": single,
        "host_cpu": model, "host_nproc": os.cpu_count(), "physical_cores": phys, "affinity_cpus": logical,
        "_check": r_all,
    }


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def build_table_image(nblocks: int, S: int = 4096) -> bytes:
    """The shim bench's SSTable image (see shim_bench): nblocks data blocks of
    S bytes, an empty metaindex, a restart-interval-1 index, the footer."""
    import ctypes
    from nvlevelz_amd import _lib
    L = _lib.lib
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
    return bytes(data)


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
    image = build_table_image(nblocks)
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
    # the same table already in HBM (nvl_sstable_verify_table_dev): only the
    # footer, index and metaindex cross PCIe
    import torch
    dimg = torch.frombuffer(bytearray(image), dtype=torch.uint8).to("cuda")
    sptr = torch.cuda.current_stream().cuda_stream

    def run_dev():
        rc = L.nvl_sstable_verify_table_dev(dimg.data_ptr(), nbytes, arr, cap, ctypes.byref(n), ctypes.byref(st),
                                            ctypes.byref(nb), sptr)
        assert rc == 0 and st.value == 0 and n.value == cap and nb.value == 0, (rc, st.value, n.value, nb.value)

    t_dev = timed(run_dev, 7)
    del dimg
    res = {"what": "nvl_sstable_verify_table on a host-resident table image (footer -> index -> every block), "
                   "wall clock per call, median",
           "table": {"data_blocks": nblocks, "block_bytes": 4096, "file_bytes": nbytes},
           "gpu": {"ms": round(t_gpu * 1e3, 3), "GiB/s": round(nbytes / t_gpu / 2**30, 3),
                   "path": "host image -> pinned staging -> H2D -> one batch kernel -> D2H"},
           "gpu_device_resident": {"ms": round(t_dev * 1e3, 3), "GiB/s": round(nbytes / t_dev / 2**30, 3),
                                   "path": "image in HBM: footer + metaindex D2H, index block parsed on "
                                           "the GPU, one batch over every block + trailer-check kernel in "
                                           "place, records D2H (nvl_sstable_verify_table_dev)"},
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


CFG5_BLOCKS = 10_000_000


def cfg5_leg(steps: int, warmup: int, rank: int, world: int, dev, red_dev, golden: dict) -> dict:
    """BASELINE config 5 beside the headline, on every `--gpus N` run (N = 1
    included): 10^7 x 4 KiB blocks IN TOTAL, round-robin over the N ranks
    (strong scaling: rank r holds global blocks r, r + N, ...; 41 GB at N = 1,
    5.1 GB per GPU at N = 8), generated in place, no data-path collective.  A
    step checksums every block of the rank once, as ONE nvl_crc32c_fixed_dev
    launch (crc32c_fixed_long_kernel from 2^18 blocks: the headline kernel's
    code under its own name, so a rocprofv3 --stats average over the whole
    command keeps the headline's launches apart).  Every rank's CRCs are
    verified before the timing (its own digest against the reference-built
    per-rank golden, then the gathered global digest: shard.verify_shards,
    tests/golden/configs.json cfg5.ranks).  Timed like the headline: barrier +
    synchronize around `steps` back-to-back launches, MAX wall time over
    ranks; the per-rank kernel period from HIP events on the launch stream."""
    import torch
    import torch.distributed as dist

    from nvlevelz_amd import crc32c, shard

    n_local = shard.local_count(CFG5_BLOCKS, rank, world)
    buf = torch.empty(max(n_local, 1) * BLOCK, dtype=torch.uint8, device=dev)
    crc32c.fill_splitmix(buf, n_local, BLOCK, SEED_CFG5, first_block=rank, block_step=world)
    stream = torch.cuda.current_stream(dev)
    out = torch.empty(max(n_local, 1), dtype=torch.int32, device=dev)
    batches = [crc32c.FixedBatch(buf, BLOCK, BLOCK, n_local, out=out[:n_local], stream=stream)] if n_local else []

    def step():
        for b in batches:
            b.launch()

    step()
    torch.cuda.synchronize()
    expect = shard.round_robin_expect(golden["cfg5"], world)
    if world > 1:
        v = shard.verify_shards(out[:n_local].to(red_dev), CFG5_BLOCKS, expect)
    else:
        v = shard.verify_local(crc32c.to_u32(out[:n_local]), expect)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    # each rank's own window (shard.timed_window: the closing barrier outside
    # `elapsed`), then the slowest rank's
    tw = shard.timed_window(step, steps, stream=stream, world=world)
    period_s = tw["period_s"]
    frac = n_local * (BLOCK + 4) / period_s / 1e9 / HBM_PEAK_GBS
    rows = shard.gather_floats([tw["elapsed_s"], period_s, tw["barrier_after_s"], n_local], red_dev)
    elapsed = float(rows[:, 0].max())
    frac_r = rows[:, 3] * (BLOCK + 4) / rows[:, 1] / 1e9 / HBM_PEAK_GBS
    frac_min = float(frac_r.min())
    nb = len(batches)
    del batches, buf, out
    torch.cuda.empty_cache()
    return {"workload": f"cfg5: 10^7 x 4 KiB blocks in total (BASELINE config 5), round-robin over {world} GPU(s), "
                        f"device-resident, generated in place",
            "value": round(CFG5_BLOCKS * BLOCK * steps / elapsed / 2**30, 3), "unit": "GiB/s",
            "scaling": "strong", "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 4), "blocks_per_gpu_max": shard.local_count(CFG5_BLOCKS, 0, world),
            "launches_per_step": nb,
            "launch_what": "a step = every block of the rank once, one nvl_crc32c_fixed_dev launch "
                           "(crc32c_fixed_long_kernel: the headline kernel's code under its own name)",
            "frac": round(frac, 4), "frac_min_over_ranks": round(frac_min, 4),
            "period_us_per_step_rank0": round(period_s * 1e6, 2),
            "frac_what": "rank 0's alg bytes (its blocks x (4096 + 4)) / its period per step (HIP events around the "
                         "timed steps / steps) / 8 TB/s; frac_min_over_ranks the slowest rank's",
            "timing_what": "value = all blocks x steps / the MAX over ranks of each rank's own elapsed (its start "
                           "after the opening barrier + synchronize to its own synchronize after the last launch; "
                           "the closing barrier is timed apart, barrier_after_ms)",
            "per_rank": _per_rank(rows),
            "traffic_over_alg": _cfg5_traffic(n_local),
            "verify": v}


def _per_rank(rows) -> list:
    """Rows of shard.gather_floats([elapsed_s, period_s, barrier_after_s,
    blocks]) -> one object per rank: its own wall window, its kernel period
    (HIP events on its launch stream) and that period's roofline fraction."""
    out = []
    for r, (el, per, bar, nb) in enumerate(rows):
        out.append({"rank": r, "elapsed_ms": round(el * 1e3, 4), "period_us": round(per * 1e6, 2),
                    "frac": round(nb * (BLOCK + 4) / per / 1e9 / HBM_PEAK_GBS, 4),
                    "barrier_after_ms": round(bar * 1e3, 4), "blocks": int(nb)})
    return out


def _cfg5_traffic(n_local: int):
    """Committed PMC (not measured in this run): HBM bytes / algorithmic bytes
    of crc32c_fixed_long_kernel over config 5's one-GPU batch
    (profiles/r05_pmc_cfg5_long.json, tools/pmc.sh + tools/pmc_workloads.py);
    None for any other per-rank batch."""
    try:
        with open(os.path.join(ROOT, "profiles", "r05_pmc_cfg5_long.json")) as f:
            w = json.load(f)["workloads"]["cfg5_one_gpu"]
        return w["traffic_over_alg"] if w["alg_bytes"] == n_local * (BLOCK + 4) else None
    except (OSError, ValueError, KeyError):
        return None


def main():
    args = parse()
    from nvlevelz_amd import launch  # (loads nothing: safe before the ranks exist)
    rc = launch.main_or_spawn(args.gpus, __file__, sys.argv[1:])
    if rc is not None:  # launcher-less N > 1: this process only waited for its N ranks
        sys.exit(rc)
    import torch
    import torch.distributed as dist

    from nvlevelz_amd import crc32c, shard

    re_ = launch.rank_env()
    world, rank, local = re_["world"], re_["rank"], re_["local_rank"]
    if world != args.gpus:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: running {world} rank(s)", file=sys.stderr)
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
        total = n_local * N
    else:
        total = 10_000_000
        n_local = (total - rank + N - 1) // N
        seed = SEED_CFG5
        workload = f"cfg5: 10^7 x 4 KiB blocks total (BASELINE config 5), round-robin over {N} GPU(s)"
        scaling = "strong"

    buf = torch.empty(n_local * BLOCK, dtype=torch.uint8, device=dev)
    crc32c.fill_splitmix(buf, n_local, BLOCK, seed, first_block=rank, block_step=N)
    stream = torch.cuda.current_stream(dev)
    batch = crc32c.FixedBatch(buf, BLOCK, BLOCK, n_local, stream=stream)  # validated once
    out = batch.out
    step = batch.launch  # one C call per step; the host stays ahead of the GPU

    step()
    torch.cuda.synchronize()

    # --- verification (untimed, before the warmup: the timed region starts
    # right after the warmup launches, not after seconds of host-side checks
    # with the GPU idle) -----------------------------------------------------
    verify = {}
    res = crc32c.to_u32(out)
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        golden = json.load(f)
    union = golden.get("cfg2_union", {}).get(str(N)) if args.config == "cfg2" and n_local == 100_000 else None
    if N > 1 and (args.config == "cfg5" or union):
        # every rank's own digest (cfg2: golden per-rank digests of the
        # weak-scaling union, global blocks 0..N*10^5-1) and the gathered
        # global digest (shard.verify_shards: ONE all_gather of the 4-byte
        # results; tests/test_dist.py drives the same function over gloo)
        g = golden["cfg5"] if args.config == "cfg5" else union
        v = shard.verify_shards(out[:n_local].to(red_dev), total, g)
        if rank == 0:
            verify.update(v)
            verify["crc0_ok"] = int(v["crc0"], 16) == golden[args.config if args.config == "cfg5" else "cfg2"][
                "crc_first"][0]
    elif args.config == "cfg5" or (N == 1 and n_local == 100_000):
        # the CRCs in global order -> digest = Value() of the little-endian
        # CRC array, golden from the reference build
        # (tests/golden/configs.json)
        g = golden[args.config]
        allc = res
        if rank == 0:
            d = crc32c.value(np.ascontiguousarray(allc, dtype="<u4").tobytes())
            verify.update({"crc0": hex(int(allc[0])), "crc0_ok": int(allc[0]) == g["crc_first"][0],
                           "crc_last_ok": int(allc[-1]) == g["crc_last"],
                           "digest": hex(d), "digest_ok": d == g["digest"], "blocks_checked": int(allc.size)})
    elif rank == 0:
        verify["crc0"] = hex(int(res[0]))
        verify["crc0_ok"] = int(res[0]) == golden["cfg2"]["crc_first"][0]

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # --- timed region ------------------------------------------------------
    # K back-to-back launches, nothing else enqueued between them.  Two HIP
    # events on the launch stream bracket the region (interval / K = mean
    # launch period, gaps included).
    K = args.steps
    tw = shard.timed_window(step, K, stream=stream, world=world)
    elapsed = tw["elapsed_s"]
    region_ms = tw["period_s"] * K * 1e3
    # Beside the in-regime figure, two untimed diagnostic passes (K launches
    # each, after the timed region; tools/rocprof_summary.py splits them off a
    # rocprofv3 trace of this command by launch order):
    #  * dispatch events: nvl_crc32c_fixed_dev_timed, whose kernel dispatch
    #    records its own start/stop events (hipExtLaunchKernel).  Back to back
    #    these overlap: a dispatch's start stamp is taken while the previous
    #    kernel still drains, so their mean can exceed the launch period and
    #    is never used for the roofline;
    #  * isolated launches: an ordinary event before and after each launch, so
    #    every launch starts from an idle queue -- what one shim call sees.
    kev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
    for e in kev:
        e.record(stream)  # materialise the HIP events
    for k in range(K):
        batch.launch_timed(kev[2 * k], kev[2 * k + 1])
    torch.cuda.synchronize()
    kern_ms = np.array([kev[2 * k].elapsed_time(kev[2 * k + 1]) for k in range(K)])
    #  * isolated launches: every launch from an idle queue (synchronize after
    #    each, as one synchronous shim call runs), an event before and after;
    #    and beside them the same K launches with their event pairs queued
    #    back to back (no synchronize): round 5's "isolated" pass, which each
    #    launch's markers slow down instead
    iso = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
    for k in range(K):
        iso[2 * k].record(stream)
        step()
        iso[2 * k + 1].record(stream)
        torch.cuda.synchronize()
    iso_ms = [iso[2 * k].elapsed_time(iso[2 * k + 1]) for k in range(K)]
    qev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
    for k in range(K):
        qev[2 * k].record(stream)
        step()
        qev[2 * k + 1].record(stream)
    torch.cuda.synchronize()
    qev_ms = [qev[2 * k].elapsed_time(qev[2 * k + 1]) for k in range(K)]
    #  * sustained: --sustained back-to-back launches (default 2000, ~0.13 s)
    #    with an event every 100, so drift from the short timed window to a
    #    long run shows as a series of segment periods
    sus = None
    if args.sustained > 0:
        seg = 100
        nseg = max(1, args.sustained // seg)
        sev = [torch.cuda.Event(enable_timing=True) for _ in range(nseg + 1)]
        sev[0].record(stream)
        for j in range(nseg):
            for _ in range(seg):
                step()
            sev[j + 1].record(stream)
        torch.cuda.synchronize()
        segs = [sev[j].elapsed_time(sev[j + 1]) * 1e3 / seg for j in range(nseg)]
        sus = {"launches": nseg * seg, "segment_launches": seg,
               "segment_period_us": [round(x, 2) for x in segs]}
    #  * the measured read ceiling on the same buffer: a plain streaming
    #    kernel (nvl_crc32c_read_probe) back to back, period by HIP events --
    #    what this box's HBM gives a read-only kernel in this very run
    probe = None
    if args.probe > 0:
        nb = (buf.numel() // 16) * 16
        sink = torch.zeros(1, dtype=torch.int32, device=dev)
        from nvlevelz_amd import _lib as nvl_lib
        lib = nvl_lib.lib
        for _ in range(50):
            assert lib.nvl_crc32c_read_probe(buf.data_ptr(), nb, sink.data_ptr(), stream.cuda_stream) == 0
        pe = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        pe[0].record(stream)
        for _ in range(args.probe):
            lib.nvl_crc32c_read_probe(buf.data_ptr(), nb, sink.data_ptr(), stream.cuda_stream)
        pe[1].record(stream)
        torch.cuda.synchronize()
        probe = {"bytes": nb, "period_us": pe[0].elapsed_time(pe[1]) * 1e3 / args.probe}
        # the same read-only kernel from an idle queue, as the isolated CRC
        # launches above: what this box's memory system gives ONE launch after
        # an idle gap (isolated calls vary 65-74 us from
        # box to box -- the ratio names the kernel's share of it)
        ip = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
        for k in range(K):
            ip[2 * k].record(stream)
            lib.nvl_crc32c_read_probe(buf.data_ptr(), nb, sink.data_ptr(), stream.cuda_stream)
            ip[2 * k + 1].record(stream)
            torch.cuda.synchronize()
        probe["isolated_median_us"] = float(np.median([ip[2 * k].elapsed_time(ip[2 * k + 1]) * 1e3 for k in range(K)]))
    # the slowest rank's own window (each rank's elapsed ends at its own
    # synchronize; the closing barrier is timed apart) and every rank's period
    rows = shard.gather_floats([elapsed, tw["period_s"], tw["barrier_after_s"], n_local], red_dev)
    own_elapsed = elapsed
    elapsed = float(rows[:, 0].max())
    total_blocks = int(round(rows[:, 3].sum()))

    value = total_blocks * BLOCK * K / elapsed / 2**30
    # Roofline: the kernel's average launch duration in the timed region
    # itself = the HIP-event interval on the launch stream / K.  Launches are
    # serialised on one stream with nothing between them, so this period
    # bounds the kernel's own duration from above (frac is a lower bound on
    # the kernel's fraction) and can never exceed the wall-clock step.
    period_s = region_ms / 1e3 / K
    step_s = elapsed / K
    assert period_s <= own_elapsed / K * 1.0001, (period_s, own_elapsed / K)  # events inside the wall-clock bracket
    alg_bytes = n_local * (BLOCK + 4)  # every input byte once + 4 B CRC out
    achieved = alg_bytes / period_s / 1e9
    frac = achieved / HBM_PEAK_GBS
    frac_wall = alg_bytes / step_s / 1e9 / HBM_PEAK_GBS  # the same over the driver-visible wall clock
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        try:
            with open(pmc) as f:
                pj = json.load(f)
            if pj.get("blocks") == n_local:
                traffic = pj.get("hbm_bytes_per_launch")
                traffic_src = pj.get("source")
        except (OSError, ValueError):
            traffic = None

    c5 = None
    if args.config == "cfg2" and args.cfg5_steps > 0:  # BASELINE config 5 beside the cfg2 headline (all ranks)
        c5 = cfg5_leg(args.cfg5_steps, args.cfg5_warmup, rank, N, dev, red_dev, golden)

    cpu = None
    e2e = None
    if rank == 0 and N == 1 and not args.no_cpu:
        host = buf[:100_000 * BLOCK].cpu().numpy() if n_local > 100_000 else buf.cpu().numpy()
        cpu = cpu_baseline(host, min(n_local, 100_000), args.cpu_seconds, args.cpu_threads)
        chk = cpu.pop("_check")
        verify["cpu_matches_gpu"] = bool(np.array_equal(chk, res[:chk.size]))
        del host
    if rank == 0 and N == 1 and not args.no_e2e:
        ne = min(n_local, 100_000)
        pinned = torch.empty(ne * BLOCK, dtype=torch.uint8).pin_memory()
        pinned.copy_(buf[:ne * BLOCK].cpu())
        hp = pinned.numpy()
        crc32c.extend_fixed_host(hp, BLOCK, BLOCK, ne)
        import resource
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t1 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            r = crc32c.extend_fixed_host(hp, BLOCK, BLOCK, ne)
        el = time.perf_counter() - t1
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        gib = ne * BLOCK * reps / 2**30
        e2e = {"value": round(gib / el, 3), "unit": "GiB/s",
               "what": f"{ne} x 4 KiB pinned host blocks -> H2D -> kernel -> D2H of u32 results "
                       f"(nvl_crc32c_fixed_host, 2-stream pipeline, synchronous), {reps} calls",
               "host_cpu_s_per_GiB": round(((ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)) / gib, 4),
               "host_cpu_what": "getrusage user + sys of every thread of this process over the calls / GiB "
                                "checksummed (the reference CPU leg: cpu_baseline.cpu_s_per_GiB)",
               "ok": bool(np.array_equal(r, res[:ne]))}

    if rank == 0:
        kern = ("crc32c_fixed_kernel<0> (aligned 4 KiB blocks, scheduler A)")
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": N,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (splitmix64 stream, SURVEY.md §8d), generated in HBM",
            "config": {"workload": workload, "blocks_per_gpu": n_local, "block_bytes": BLOCK,
                       "parallelism": f"{N} independent shard(s), no data-path collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(frac, 4), "traffic": traffic,
                         "traffic_source": (f"committed PMC, not measured in this run: profiles/pmc_traffic.json "
                                            f"({traffic_src}; rocprofv3 --pmc passes over this kernel and batch: "
                                            f"L2 memory-side request counts by size, FETCH_SIZE x 2 / WRITE_SIZE "
                                            f"beside, per MI355X_MICROARCH.md § HBM)"
                                            if traffic is not None else None),
                         "kernel": kern, "alg_bytes_per_launch": alg_bytes,
                         "mean_kernel_us": round(period_s * 1e6, 2),
                         "kernel_what": "average launch duration over the K timed launches: HIP events recorded on "
                                        "the launch stream around the timed region / K (back-to-back launches, "
                                        "nothing else enqueued; an upper bound on the kernel's own time); "
                                        "achieved = alg_bytes / this",
                         "frac_wall": round(frac_wall, 4),
                         "frac_wall_what": "alg_bytes / ms_per_step (wall clock incl. synchronize) / peak",
                         "dispatch_event_mean_us": round(float(kern_ms.mean()) * 1e3, 2),
                         "dispatch_event_what": "untimed diagnostic: start/stop events recorded by each kernel "
                                                "dispatch (hipExtLaunchKernel), K back-to-back launches; they overlap "
                                                "the previous kernel's drain, so not used for frac",
                         "isolated_median_us": round(float(np.median(iso_ms)) * 1e3, 2),
                         "isolated_frac": round(alg_bytes / (float(np.median(iso_ms)) / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                         "isolated_what": "untimed diagnostic: ordinary events before and after each launch and a "
                                          "synchronize after it (every launch starts from an idle queue, as a single "
                                          "synchronous shim call does); median",
                         "queued_event_pairs_median_us": round(float(np.median(qev_ms)) * 1e3, 2),
                         "queued_event_pairs_what": "untimed diagnostic: the same K launches with their event pairs "
                                                    "queued back to back, no synchronize between them (round 5's "
                                                    "isolated pass): each launch's start waits on the markers of "
                                                    "the one before (DESIGN.md section 4)"},
            "timing": {"what": "value = all ranks' blocks x K / the MAX over ranks of each rank's own elapsed "
                               "(from its start after the opening barrier + synchronize to its own synchronize "
                               "after the K launches); the closing barrier is outside it (barrier_after_ms); "
                               "per_rank: each rank's window, its kernel period (HIP events on its launch "
                               "stream / K) and that period's roofline fraction",
                       "per_rank": _per_rank(rows)},
            "cpu_baseline": cpu,
            "verify": verify,
        }
        if sus:
            mp = float(np.mean(sus["segment_period_us"]))
            sus.update({"mean_period_us": round(mp, 2), "frac": round(alg_bytes / (mp * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                        "first_segment_frac": round(alg_bytes / (sus["segment_period_us"][0] * 1e-6) / 1e9 /
                                                    HBM_PEAK_GBS, 4),
                        "last_segment_frac": round(alg_bytes / (sus["segment_period_us"][-1] * 1e-6) / 1e9 /
                                                   HBM_PEAK_GBS, 4),
                        "what": "untimed diagnostic after the timed region: back-to-back launches, HIP events every "
                                "100; frac over the whole run (the timed window's frac is roofline.frac)"})
            line["roofline"]["sustained"] = sus
        if probe:
            cg = probe["bytes"] / (probe["period_us"] * 1e-6) / 1e9
            line["roofline"]["read_ceiling"] = {
                "period_us": round(probe["period_us"], 2), "achieved": round(cg, 1), "unit": "GB/s",
                "frac_of_peak": round(cg / HBM_PEAK_GBS, 4), "kernel_over_ceiling": round(achieved / cg, 4),
                "what": "untimed diagnostic: nvl_crc32c_read_probe (a read-only streaming kernel, four 16-byte "
                        "nontemporal loads in flight per thread, 256 x 1024) back to back over the same buffer on "
                        "the same box, %d launches after 50, run after the sustained pass; kernel_over_ceiling = "
                        "roofline.achieved / this rate (the short timed window, which still ramps); "
                        "sustained_over_ceiling = the same for roofline.sustained's mean period, both ramped "
                        "(DESIGN.md section 4)" % args.probe}
            line["roofline"]["read_ceiling"]["isolated_period_us"] = round(probe["isolated_median_us"], 2)
            line["roofline"]["read_ceiling"]["isolated_kernel_over_ceiling"] = round(
                probe["isolated_median_us"] / (float(np.median(iso_ms)) * 1e3), 4)
            line["roofline"]["read_ceiling"]["isolated_what"] = (
                "the read-only probe launched from an idle queue like isolated_median_us (event before and "
                "after, synchronize between launches; median of K): isolated_kernel_over_ceiling = its "
                "period / the CRC kernel's isolated median -- the share of an isolated call's time the memory "
                "system's idle-to-busy ramp alone accounts for (DESIGN.md section 4)")
            if sus:
                line["roofline"]["read_ceiling"]["sustained_over_ceiling"] = round(
                    alg_bytes / (sus["mean_period_us"] * 1e-6) / 1e9 / cg, 4)
        if c5:
            line["cfg5"] = c5
        if e2e:
            line["e2e"] = e2e
        if args.shims and N == 1:
            line["shims"] = shim_bench()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
