"""Per-step cost of back-to-back config-2 launches: plain loop (wall clock),
loop with an event between launches (bench.py's roofline pass), and the same
K launches replayed from a captured graph."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import crc32c

dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
crc32c.init(0)
n, L = 100000, 4096
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
crc32c.fill_splitmix(buf, n, L, 0x5EED0001)
K = int(os.environ.get("K", "300"))


def plain(step, st):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize(); return (time.perf_counter() - t0) / K * 1e6


def with_events(step, st):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    torch.cuda.synchronize(); t0 = time.perf_counter()
    ev[0].record(st)
    for k in range(K):
        step(); ev[k + 1].record(st)
    torch.cuda.synchronize(); w = (time.perf_counter() - t0) / K * 1e6
    d = [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(K)]
    return w, float(np.mean(d))


st = torch.cuda.Stream(dev)
with torch.cuda.stream(st):
    batch = crc32c.FixedBatch(buf, L, L, n, stream=st)
    for _ in range(50):
        batch.launch()
    for r in range(3):
        print(f"round {r}: plain {plain(batch.launch, st):.2f} us/step; events wall/mean "
              + "%.2f / %.2f us" % with_events(batch.launch, st))
    g = torch.cuda.CUDAGraph()
    G = 50
    with torch.cuda.graph(g, stream=st):
        for _ in range(G):
            batch.launch()
    g.replay(); torch.cuda.synchronize()
    for r in range(3):
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(K // G):
            g.replay()
        torch.cuda.synchronize()
        print(f"graph round {r}: {(time.perf_counter() - t0) / (K // G * G) * 1e6:.2f} us/step")
    ref = crc32c.to_u32(batch.out).copy()
    batch.out.zero_(); g.replay(); torch.cuda.synchronize()
    print("graph output identical:", bool(np.array_equal(ref, crc32c.to_u32(batch.out))))
