"""Multi-GPU sharding of independent blocks.

Every block's CRC is independent, so a batch shards across the GPUs of a node
with no data-path exchange: buffer i lives on (and is checksummed by) rank
i mod G (BASELINE config 5, "round-robin").  The only collective is the
optional gather of the 4-byte results to one rank, done with
torch.distributed (RCCL over xGMI on the GPU box, gloo in the CPU tests) in
ONE all_gather of equal-size slices -- never per block.
"""
from __future__ import annotations

import numpy as np

# (timed_window / gather_floats: bench.py's per-rank timing, SURVEY §8e "wall
# time from the first launch to the last completion" -- the slowest rank's)


def local_count(n_total: int, rank: int, world: int) -> int:
    """Number of round-robin blocks rank owns out of n_total."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    return (n_total - rank + world - 1) // world if n_total > rank else 0


def local_ids(n_total: int, rank: int, world: int) -> np.ndarray:
    """Global block ids owned by rank: rank, rank+G, rank+2G, ..."""
    return np.arange(rank, n_total, world, dtype=np.int64)


def interleave(parts, n_total: int) -> np.ndarray:
    """Inverse of the round-robin split: parts[r] holds rank r's CRCs in local order."""
    world = len(parts)
    out = np.empty(n_total, dtype=np.uint32)
    for r, p in enumerate(parts):
        p = np.asarray(p, dtype=np.uint32)
        assert p.size == local_count(n_total, r, world)
        out[r::world] = p
    return out


def gather_crcs(local, n_total: int, group=None):
    """All-gather every rank's CRC slice (int32 tensor, round-robin order) and
    return the global u32 array in block order on every rank.

    Slices are padded to a common length so the exchange is one all_gather
    call (bucketed: 4 bytes per block, e.g. 40 MB for 10^7 blocks)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    per = local_count(n_total, 0, world)  # rank 0 owns the most
    buf = torch.zeros(per, dtype=torch.int32, device=local.device)
    buf[:local.numel()] = local
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf, group=group)
    parts = [o[:local_count(n_total, r, world)].cpu().numpy().view(np.uint32) for r, o in enumerate(outs)]
    return interleave(parts, n_total)


def digest(crcs: np.ndarray) -> int:
    """crc32c::Value over the little-endian u32 array (SURVEY.md §8d digest),
    computed with the engine's host path."""
    from . import crc32c
    return crc32c.value(np.ascontiguousarray(crcs, dtype="<u4").view(np.uint8))


def round_robin_expect(entry: dict, world: int) -> dict:
    """verify_shards' expectations for `world` ranks from a golden entry of a
    round-robin batch: the global "digest" / "crc_last", and each rank's own
    digest from entry["ranks"][str(world)]["rank_digests"] (config 5,
    tests/golden/configs.json; at world 1 the rank digest is the digest)."""
    exp = {"digest": entry["digest"]}
    if "crc_last" in entry:
        exp["crc_last"] = entry["crc_last"]
    if world == 1:
        exp["rank_digests"] = [entry["digest"]]
    else:
        r = entry.get("ranks", {}).get(str(world))
        if r is not None:
            exp["rank_digests"] = list(r["rank_digests"])
    return exp


def verify_local(crcs: np.ndarray, expect: dict) -> dict:
    """verify_shards' report for one rank holding the whole batch (N = 1, no
    process group)."""
    d = digest(crcs)
    out = {"rank_digests_ok": d == expect["rank_digests"][0] if expect.get("rank_digests") else None,
           "digest": hex(d), "digest_ok": d == expect["digest"], "blocks_checked": int(crcs.size),
           "crc0": hex(int(crcs[0])) if crcs.size else None}
    if "crc_last" in expect and crcs.size:
        out["crc_last_ok"] = int(crcs[-1]) == expect["crc_last"]
    return out


def timed_window(launch, steps: int, *, stream=None, world: int = 1, sync=None, group=None) -> dict:
    """One rank's timed region (bench.py's contract: barrier + synchronize on
    both sides of exactly `steps` launches).  Returns this rank's own
    `elapsed_s` -- from its start (after the opening barrier and
    synchronize) to its own synchronize after the last launch -- and, apart
    from it, `barrier_after_s`: the time this rank then waits in the closing
    barrier for the slowest rank.  The closing barrier stays outside
    `elapsed_s`, so the max over ranks of `elapsed_s` (max_over_ranks) is the
    slowest rank's own time, not that time plus an RCCL barrier's latency and
    the other ranks' skew (the 20-launch windows are
    ~1.3 ms, where a barrier's tens of µs read as a false efficiency loss).
    With `stream`, two HIP events on it bracket the launches: `period_s` =
    their interval / steps (the per-rank kernel period).  `sync` (default
    torch.cuda.synchronize) lets CPU tests time host-side work."""
    import time

    import torch
    import torch.distributed as dist

    if sync is None:
        sync = torch.cuda.synchronize
    ev = None
    if stream is not None:
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if world > 1:
        dist.barrier(group=group)
    sync()
    t0 = time.perf_counter()
    if ev:
        ev[0].record(stream)
    for _ in range(steps):
        launch()
    if ev:
        ev[1].record(stream)
    sync()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier(group=group)
    t2 = time.perf_counter()
    out = {"elapsed_s": t1 - t0, "barrier_after_s": t2 - t1, "period_s": None}
    if ev:
        out["period_s"] = ev[0].elapsed_time(ev[1]) / 1e3 / max(steps, 1)
    return out


def gather_floats(vals, device, group=None) -> np.ndarray:
    """All-gather a short float vector from every rank: row r = rank r's
    (float64; one all_gather, outside any timed region).  Without a process
    group, the one row."""
    import torch
    import torch.distributed as dist

    v = torch.tensor([float(x) for x in vals], dtype=torch.float64, device=device)
    if not (dist.is_available() and dist.is_initialized()):
        return v.cpu().numpy()[None, :]
    outs = [torch.empty_like(v) for _ in range(dist.get_world_size(group))]
    dist.all_gather(outs, v, group=group)
    return torch.stack(outs).cpu().numpy()


def verify_shards(local, n_total: int, expect: dict, group=None) -> dict:
    """Check every rank's CRCs of a round-robin batch (outside any timed
    region).  local: this rank's int32 CRC tensor in local order; expect:
    a golden entry with "digest" (over all n_total CRCs in global order) and,
    optionally, "rank_digests" (each rank's own digest over its blocks in
    local order) and "crc_last".  Every rank checks its own digest (the
    verdicts are AND-reduced, so rank 0 learns about every rank), then the
    slices are all-gathered (gather_crcs) and the global digest checked.
    Returns the same dict on every rank."""
    import torch
    import torch.distributed as dist

    rank = dist.get_rank(group)
    mine = local.detach().cpu().numpy().view(np.uint32)
    rd = expect.get("rank_digests")
    own_ok = rd is not None and rank < len(rd) and digest(mine) == rd[rank]
    flag = torch.tensor([1 if own_ok else 0], dtype=torch.int32, device=local.device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    full = gather_crcs(local, n_total, group)
    d = digest(full)
    out = {"rank_digests_ok": bool(flag.item()) if rd is not None else None,
           "digest": hex(d), "digest_ok": d == expect["digest"], "blocks_checked": int(full.size),
           "crc0": hex(int(full[0])) if full.size else None}
    if "crc_last" in expect and full.size:
        out["crc_last_ok"] = int(full[-1]) == expect["crc_last"]
    return out
