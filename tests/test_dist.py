"""Round-robin sharding + result gather over torch.distributed, world_size 2
on the CPU (gloo).  On the GPU box the same code runs over RCCL; per-rank
checksums there come from the HIP kernels -- here the checker computes them,
so this exercises the partition, the single all_gather and the reassembly."""
import os
import socket

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
    from nvlevelz_amd import shard
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
        local = p.fixed(buf, L, L, ids.size) if ids.size else np.zeros(0, dtype=np.uint32)
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
