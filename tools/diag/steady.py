"""Back-to-back launches of the config-2 fast path: per-launch duration trend
(events, queue kept full), to see clock/power behaviour over time."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
from nvlevelz_amd import _lib
lib = _lib.lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
n, L = 100000, 4096
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
out = torch.empty(n, dtype=torch.int32, device=dev)
st = torch.cuda.current_stream().cuda_stream
f = lib.nvl_crc32c_fixed_dev
bp, op = buf.data_ptr(), out.data_ptr()
K = int(os.environ.get("K", "3000"))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
torch.cuda.synchronize()
t0 = time.perf_counter()
ev[0].record()
for k in range(K):
    f(bp, L, L, n, None, 0, op, 0, None, 0, st)
    ev[k + 1].record()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
d = np.array([ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(K)])
print(f"wall {wall*1e3:.1f} ms for {K} launches -> {wall/K*1e6:.1f} us/launch")
for i in range(0, K, K // 15):
    seg = d[i:i + K // 15]
    print(f"launch {i:5d}-{i+len(seg):5d}: median {np.median(seg):6.1f} us  min {seg.min():6.1f}  max {seg.max():6.1f}")
