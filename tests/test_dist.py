"""Round-robin sharding + result gather over torch.distributed, world_size 2
and 3 on the CPU (gloo).  On the GPU box the same code runs over RCCL with
per-rank checksums from the HIP kernels; here every rank checksums its shard
with the engine's host path (libnvl_crc32c.so nvl_crc32c_value) and the
oracle only checks the reassembled result.

test_spawned_ranks_*: the launcher-less path of ``bench.py --gpus N``
(nvlevelz_amd.launch.spawn_ranks, no torchrun) with tests/dist_rank_worker.py
as the rank body: 2 ranks reassemble BASELINE config 2's golden digest."""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import load_golden

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, result_q):
    import torch.distributed as dist
    import oracle
    from nvlevelz_amd import crc32c, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = oracle.port()
        L = 4096
        ids = shard.local_ids(n, rank, world)
        assert ids.size == shard.local_count(n, rank, world)
        # this rank's resident shard: block k = global block ids[k] of the stream
        buf = np.concatenate([p.fill(0x5EED0001, int(i) * L, L) for i in ids]) if ids.size else \
            np.zeros(0, dtype=np.uint8)
        # the engine's host path (the reference's Value() replacement), block by block
        local = np.array([crc32c.value(buf[k * L:(k + 1) * L]) for k in range(ids.size)], dtype=np.uint32)
        t = torch.from_numpy(local.view(np.int32).copy())
        full = shard.gather_crcs(t, n)
        result_q.put((rank, full.tolist(), shard.digest(full)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (2, 999), (3, 10), (2, 1)])
def test_round_robin_gather_matches_single_process(world, n):
    import torch.multiprocessing as mp
    import oracle
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    p = oracle.port()
    whole = p.fixed(p.fill(0x5EED0001, 0, n * 4096), 4096, 4096, n)
    for rank, full, dg in res:
        assert full == whole.tolist()
        assert dg == p.digest(whole)
    if n == 1000:
        g = load_golden("configs")["cfg2"]
        assert whole[:8].tolist() == g["crc_first"]


def _verify_worker(rank, world, port, per, expect, result_q):
    """One rank of bench.py's N > 1 verification (shard.verify_shards) on the
    CPU: rank r checksums its round-robin shard (global blocks r, r+N, ...,
    `per` of them) with the engine's host path and verifies it."""
    import torch.distributed as dist
    import oracle
    from nvlevelz_amd import crc32c, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        L = 4096
        n = per * world
        whole = oracle.port().fill(0x5EED0001, 0, n * L).reshape(n, L)
        mine = np.ascontiguousarray(whole[rank::world])
        del whole
        local = np.array([crc32c.value(mine[k]) for k in range(per)], dtype=np.uint32)
        if rank == 1 and expect.get("corrupt_rank1"):
            local[per // 2] ^= 1
        v = shard.verify_shards(torch.from_numpy(local.view(np.int32).copy()), n, expect)
        result_q.put((rank, v))
    finally:
        dist.destroy_process_group()


def _run_verify(world, per, expect):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_verify_worker, args=(r, world, port, per, expect, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    return res


def test_verify_shards_cfg2_union_world2():
    """bench.py --gpus 2's verification on the weak-scaling union (2 x 10^5
    blocks): both ranks' own digests and the gathered digest equal the
    reference-built goldens (tests/golden/configs.json cfg2_union)."""
    g = load_golden("configs")["cfg2_union"]["2"]
    res = _run_verify(2, 100_000, g)
    for r, v in res.items():
        assert v["rank_digests_ok"] is True and v["digest_ok"] is True and v["crc_last_ok"] is True, (r, v)
        assert v["blocks_checked"] == 200_000


@pytest.mark.parametrize("corrupt", [False, True])
def test_verify_shards_world3(corrupt):
    """World size 3 (no golden: expectations from the oracle); one flipped
    CRC on rank 1 fails rank 1's own digest, which every rank then reports
    (AND-reduced), and the global digest."""
    import oracle
    p = oracle.port()
    per, world = 700, 3
    n = per * world
    whole = p.fixed(p.fill(0x5EED0001, 0, n * 4096), 4096, 4096, n)
    exp = {"digest": p.digest(whole), "crc_last": int(whole[-1]),
           "rank_digests": [p.digest(whole[r::world]) for r in range(world)], "corrupt_rank1": corrupt}
    res = _run_verify(world, per, exp)
    for r, v in res.items():
        assert v["rank_digests_ok"] is (not corrupt), (r, v)
        assert v["digest_ok"] is (not corrupt), (r, v)


def _cfg5_worker(rank, world, port, n, entry, result_q):
    """One rank of bench.py's cfg5 leg on the CPU: rank r's round-robin shard
    of the config-5 stream (seed 0x5EED0005, global blocks r, r + N, ... as
    fill_splitmix(first_block=r, block_step=N) lays them out), checksummed
    by the engine's host path, verified with the leg's own expectations
    (shard.round_robin_expect over a golden-shaped entry)."""
    import torch.distributed as dist
    import oracle
    from nvlevelz_amd import crc32c, shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p, L = oracle.port(), 4096
        ids = shard.local_ids(n, rank, world)
        local = np.array([crc32c.value(p.fill(0x5EED0005, int(i) * L, L)) for i in ids], dtype=np.uint32)
        v = shard.verify_shards(torch.from_numpy(local.view(np.int32).copy()), n,
                                shard.round_robin_expect(entry, world))
        result_q.put((rank, v))
    finally:
        dist.destroy_process_group()


def test_cfg5_leg_partition_and_verify_world2():
    """bench.py's cfg5 leg at --gpus 2 (strong scaling: the batch's blocks
    split round-robin, 10^7 on the GPU box; here the first 3001 blocks of the
    same stream): both ranks' own digests and the gathered digest pass, with
    the expectations in the golden's shape (cfg5.ranks[N].rank_digests)."""
    import torch.multiprocessing as mp
    import oracle
    p = oracle.port()
    n, world = 3001, 2
    whole = p.fixed(p.fill(0x5EED0005, 0, n * 4096), 4096, 4096, n)
    g = load_golden("configs")["cfg5"]
    assert whole[:8].tolist() == g["crc_first"]  # the same stream as the golden's
    entry = {"digest": p.digest(whole), "crc_last": int(whole[-1]),
             "ranks": {str(world): {"rank_digests": [p.digest(whole[r::world]) for r in range(world)]}}}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cfg5_worker, args=(r, world, port, n, entry, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for r, v in res.items():
        assert v["rank_digests_ok"] is True and v["digest_ok"] is True and v["crc_last_ok"] is True, (r, v)
        assert v["blocks_checked"] == n


def test_cfg5_golden_rank_expectations():
    """The cfg5 golden carries per-rank digests for every N the driver runs
    (bench.py --gpus 1/2/4/8, plus 3); at N = 1 the rank digest is the digest;
    verify_local reproduces the N = 1 report on a small batch."""
    from nvlevelz_amd import shard
    import oracle
    g = load_golden("configs")["cfg5"]
    for N in (1, 2, 3, 4, 8):
        e = shard.round_robin_expect(g, N)
        assert e["digest"] == g["digest"] and e["crc_last"] == g["crc_last"]
        assert len(e["rank_digests"]) == N
    p = oracle.port()
    whole = p.fixed(p.fill(0x5EED0005, 0, 64 * 4096), 4096, 4096, 64)
    e = {"digest": p.digest(whole), "crc_last": int(whole[-1]), "rank_digests": [p.digest(whole)]}
    v = shard.verify_local(whole, e)
    assert v["digest_ok"] and v["rank_digests_ok"] and v["crc_last_ok"]
    whole[3] ^= 1
    assert not shard.verify_local(whole, e)["digest_ok"]


def test_partition_math():
    from nvlevelz_amd import shard
    for n in (0, 1, 7, 100000, 10_000_000):
        for world in (1, 2, 3, 8):
            counts = [shard.local_count(n, r, world) for r in range(world)]
            assert sum(counts) == n
            assert max(counts) - min(counts) <= 1
            ids = np.concatenate([shard.local_ids(n, r, world) for r in range(world)]) if n else []
            assert sorted(ids) == list(range(n))
    parts = [np.arange(0, 10, 3), np.arange(1, 10, 3), np.arange(2, 10, 3)]
    assert shard.interleave(parts, 10).tolist() == list(range(10))


WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dist_rank_worker.py")


def _spawn(n_ranks, args, timeout=300):
    """Run the rank worker through launch.spawn_ranks in a fresh interpreter
    (as bench.py's parent would: no torchrun, no WORLD_SIZE)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    code = ("import sys; sys.path.insert(0, %r); from nvlevelz_amd import launch; "
            "sys.exit(launch.spawn_ranks(%d, [sys.executable, '-u', %r] + %r, grace_s=5.0))"
            % (os.path.dirname(os.path.dirname(WORKER)), n_ranks, WORKER, [str(a) for a in args]))
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=timeout)
    return r, time.monotonic() - t0


def test_spawned_ranks_reassemble_cfg2_digest():
    g = load_golden("configs")["cfg2"]
    r, _ = _spawn(2, [100_000, hex(g["digest"])])
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("digest %#010x" % g["digest"]) == 2, r.stdout


def test_spawned_ranks_small_world3():
    import oracle
    p = oracle.port()
    n = 1001
    whole = p.fixed(p.fill(0x5EED0001, 0, n * 4096), 4096, 4096, n)
    r, _ = _spawn(3, [n, hex(p.digest(whole))])
    assert r.returncode == 0, r.stdout + r.stderr


def test_spawned_rank_failure_stops_the_others():
    # rank 1 exits 7 before the rendezvous; rank 0 would wait in
    # init_process_group for 30 minutes unless the spawner stops it
    r, el = _spawn(2, [16, "0x0", 1], timeout=120)
    assert r.returncode == 7, r.stdout + r.stderr
    assert el < 60


def test_launch_module_loads_no_hip():
    """The spawner's parent must not touch a GPU: importing the launch module
    (and the package) loads neither libnvl_crc32c.so nor torch."""
    code = ("import sys; sys.path.insert(0, %r); import nvlevelz_amd.launch as l; "
            "print(int(l.rank_env()['world'])); "
            "print(any('nvl_crc32c' in m or m == 'torch' for m in sys.modules)); "
            "import os; print(any('libnvl_crc32c' in x for x in open('/proc/self/maps').read().split()))"
            % os.path.dirname(os.path.dirname(WORKER)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["1", "False", "False"], r.stdout


def _window_worker(rank, world, port, result_q):
    """bench.py's timed region on the CPU (shard.timed_window, gloo): rank 1's
    launches take 60 ms each, rank 0's 1 ms, so rank 0 finishes early and
    waits in the closing barrier."""
    import torch.distributed as dist
    from nvlevelz_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dt = 0.060 if rank == 1 else 0.001
        tw = shard.timed_window(lambda: time.sleep(dt), 4, world=world, sync=lambda: None)
        rows = shard.gather_floats([tw["elapsed_s"], 1.0, tw["barrier_after_s"], 10], torch.device("cpu"))
        result_q.put((rank, tw, rows.tolist()))
    finally:
        dist.destroy_process_group()


def test_timed_window_keeps_the_closing_barrier_outside_elapsed():
    """each rank's `elapsed` ends at its own synchronize;
    the wait for the slowest rank is reported apart (barrier_after_s), and the
    line's time is the max over ranks of the ranks' own windows."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_window_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = {r: (tw, rows) for r, tw, rows in (q.get(timeout=120) for _ in range(2))}
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    tw0, rows = res[0]
    tw1, _ = res[1]
    assert tw0["period_s"] is None  # no stream: no events
    assert tw0["elapsed_s"] < 0.1, tw0          # 4 x 1 ms of its own work
    assert tw0["barrier_after_s"] > 0.1, tw0    # then waits ~240 ms for rank 1, outside elapsed
    assert 0.23 < tw1["elapsed_s"] < 1.0, tw1
    assert res[1][1] == rows                    # every rank holds every rank's row
    assert max(r[0] for r in rows) == tw1["elapsed_s"]
    assert [r[3] for r in rows] == [10.0, 10.0]


def test_timed_window_single_rank():
    from nvlevelz_amd import shard
    calls = []
    tw = shard.timed_window(lambda: calls.append(1), 5, sync=lambda: None)
    assert len(calls) == 5 and tw["barrier_after_s"] < 0.01 and tw["period_s"] is None
    rows = shard.gather_floats([tw["elapsed_s"], 2.0], torch.device("cpu"))
    assert rows.shape == (1, 2) and rows[0, 1] == 2.0
