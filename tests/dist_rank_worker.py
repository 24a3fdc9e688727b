"""One rank of the launcher-less multi-rank path, on the CPU (gloo).

Started N times by nvlevelz_amd.launch.spawn_ranks from
tests/test_dist.py::test_spawned_ranks_reassemble_cfg2_digest -- the same
spawner and the same shard.gather_crcs that ``bench.py --gpus N`` uses --
with RANK/WORLD_SIZE/MASTER_* in the environment and no torchrun.  Rank r
holds the round-robin shard r, r+N, ... of BASELINE config 2's blocks
(SURVEY.md §8d stream, made by the oracle's generator: test data), checksums
it with the engine's host path (libnvl_crc32c.so nvl_crc32c_value, the
reference's Value() replacement), all-gathers the 4-byte results and checks
the reassembled digest on every rank.

    python tests/dist_rank_worker.py N_BLOCKS EXPECT_DIGEST [FAIL_RANK]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    n = int(sys.argv[1])
    expect = int(sys.argv[2], 0)
    fail_rank = int(sys.argv[3]) if len(sys.argv) > 3 else -1
    import numpy as np
    import torch
    import torch.distributed as dist

    import oracle  # the synthetic stream's generator (test data only)
    from nvlevelz_amd import crc32c, launch, shard

    env = launch.rank_env()
    rank, world = env["rank"], env["world"]
    if rank == fail_rank:
        return 7  # a rank that fails before the rendezvous: the spawner must stop the others
    dist.init_process_group("gloo")
    try:
        assert dist.get_world_size() == world and dist.get_rank() == rank
        L = 4096
        whole = oracle.port().fill(0x5EED0001, 0, n * L).reshape(n, L)
        mine = np.ascontiguousarray(whole[rank::world])  # round-robin shard: global ids rank, rank+N, ...
        del whole
        assert mine.shape[0] == shard.local_count(n, rank, world)
        crcs = np.array([crc32c.value(mine[k]) for k in range(mine.shape[0])], dtype=np.uint32)
        full = shard.gather_crcs(torch.from_numpy(crcs.view(np.int32).copy()), n)
        d = shard.digest(full)
        print(f"rank {rank}/{world}: {mine.shape[0]} blocks, digest {d:#010x}", flush=True)
        return 0 if d == expect else 3
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
