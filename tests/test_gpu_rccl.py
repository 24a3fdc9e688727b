"""The RCCL branch of the N-rank path on one GPU (VERDICT r03, weak 1 gap 2).

bench.py initialises `init_process_group("nccl", device_id=dev)` only when
WORLD_SIZE > 1, and the container has no GPU, so the multi-rank tests run over
gloo.  Here one rank initialises the nccl (= RCCL) backend for real on the
box's GPU, computes config 2 through the HIP engine, and runs what the N-rank
bench runs over RCCL: `shard.verify_shards` (AND-reduce + all_gather of the
CRCs on device tensors), the MAX all_reduce of the step time, a barrier.
World size 1 is what one GPU allows (RCCL refuses two ranks on one device);
the gather / reduce code paths are the N-rank ones.  The rank is a child
process (its own rendezvous on 127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

SCRIPT = r"""
import json, os, sys
import torch, torch.distributed as dist
sys.path.insert(0, os.environ["NVL_ROOT"])
from nvlevelz_amd import crc32c, shard
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", device_id=dev)
crc32c.init(0)
g = json.load(open(os.path.join(os.environ["NVL_ROOT"], "tests", "golden", "configs.json")))["cfg2"]
n, L = g["n"], g["len"]
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
crc32c.fill_splitmix(buf, n, L, g["seed"], first_block=0, block_step=1)
batch = crc32c.FixedBatch(buf, L, L, n, stream=torch.cuda.current_stream(dev))
batch.launch()
torch.cuda.synchronize()
v = shard.verify_shards(batch.out[:n], n, g)
t = torch.tensor([0.0625], device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
dist.barrier()
print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(), "max": float(t.item()), **v}),
      flush=True)
dist.destroy_process_group()
"""


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gpus() -> int:
    import torch
    return torch.cuda.device_count()  # (counts without initialising HIP in this process)


@pytest.mark.gpu
@pytest.mark.skipif(_gpus() == 0, reason="no GPU")
def test_rccl_rank_path_one_gpu():
    env = dict(os.environ, NVL_ROOT=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0",
               LOCAL_RANK="0", WORLD_SIZE="1")
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["backend"] == "nccl" and d["world"] == 1
    assert d["digest_ok"] and d["crc_last_ok"] and d["blocks_checked"] == 100_000
    assert d["max"] == 0.0625
