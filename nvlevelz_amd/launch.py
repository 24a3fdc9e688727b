"""One process per GPU without a launcher.

``bench.py --gpus N`` run without torch.distributed.run starts its N ranks
through :func:`spawn_ranks`: N child processes of the same command, each with
RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT
set as torchrun would set them (rendezvous on 127.0.0.1).  The parent never
touches a GPU -- this module imports nothing that loads HIP -- and never
re-execs itself: it only waits for the children and returns the first
non-zero exit status.  A rank that fails makes the parent stop the others
(SIGTERM to their PIDs, then SIGKILL after a grace period).

:func:`rank_env` reads the same variables back inside a rank.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind((host, 0))
        return so.getsockname()[1]


def rank_envs(n: int, port: int, base: Optional[Dict[str, str]] = None) -> List[Dict[str, str]]:
    """The environment of each of n ranks (torchrun's variable names)."""
    if n < 1:
        raise ValueError("need at least one rank")
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL)
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def spawn_ranks(n: int, cmd: Sequence[str], *, env: Optional[Dict[str, str]] = None, grace_s: float = 20.0,
                poll_s: float = 0.05) -> int:
    """Run ``cmd`` as n ranks and wait for all of them.

    Returns 0 when every rank exits 0, else the first non-zero status seen
    (a negative value is a signal, as in subprocess).  No rank outlives the
    call: after the first failure the rest get SIGTERM, and SIGKILL once
    ``grace_s`` has passed."""
    port = free_port()
    procs = [subprocess.Popen(list(cmd), env=e) for e in rank_envs(n, port, env)]
    rc = 0
    live = list(procs)
    deadline = None
    try:
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in live:
                        q.send_signal(signal.SIGTERM)
                    deadline = time.monotonic() + grace_s
            if deadline is not None and time.monotonic() > deadline:
                for q in live:
                    q.kill()
                deadline = None
            time.sleep(poll_s)
    finally:
        for q in procs:  # (an exception in the parent: stop the ranks by PID)
            if q.poll() is None:
                q.kill()
                q.wait()
    return rc


def rank_env() -> Dict[str, int]:
    """(rank, local_rank, world) of this process; a single rank without a launcher."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if not 0 <= rank < world:
        raise ValueError(f"RANK={rank} outside WORLD_SIZE={world}")
    return {"rank": rank, "local_rank": local, "world": world}


def main_or_spawn(n: int, script: str, argv: Sequence[str]) -> Optional[int]:
    """In a launcher-less parent with n > 1: spawn the ranks of ``script argv``
    and return their status.  Inside a rank (WORLD_SIZE set) or for n == 1:
    None (the caller runs its rank body)."""
    if n > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(n, [sys.executable, "-u", os.path.abspath(script)] + list(argv))
    return None
