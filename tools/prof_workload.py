"""Fixed workloads for rocprofv3 counter passes and kernel traces, K launches each.
    python3 tools/prof_workload.py [--lib build/libnvl_crc32c_X.so] [--config cfg2|cfg3|var4097]
                                   [--blocks N] [--launches K]
cfg2:    N x 4096 B fixed stride (fast path, nvl_crc32c_fixed_dev)
cfg3:    BASELINE config 3 (1 GiB, 32672 buffers of 512 B..64 KiB packed back to back, nvl_crc32c_batch_dev)
var4097: N buffers of 4097 B at stride 4101 -- the whole-table verify shape (block | type, then the
         4-byte stored CRC), through nvl_crc32c_batch_dev
gen:     N x 4096 B at stride 4099 from an odd base (fixed-stride general path)
rand:    N buffers of 3364..4109 B at stride length+4 (data blocks at block_size 4096), batch_dev
(batch_dev routes: a region-shaped batch runs plan + route kernel (region path) + the body kernel's early
exit; --shuffle makes it not region-shaped, so the route kernel runs the head kernel's work)
"""
import argparse, ctypes, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from nvlevelz_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None); ap.add_argument("--blocks", type=int, default=100000)
ap.add_argument("--launches", type=int, default=20); ap.add_argument("--len", type=int, default=4096)
ap.add_argument("--config", default="cfg2", choices=["cfg2", "cfg3", "var4097", "gen", "rand", "varlen"])
ap.add_argument("--gap", type=int, default=4)  # varlen: bytes between buffers
ap.add_argument("--region", action="store_true", help="variable configs through nvl_crc32c_region_dev")
ap.add_argument("--shaped", action="store_true", help="with --region: NVL_CRC32C_FLAG_REGION_SHAPED (one launch)")
ap.add_argument("--shuffle", action="store_true", help="variable configs in a random order (not region-shaped: "
                                                       "the routed call runs the batch kernels)")
ap.add_argument("--copies", type=int, default=1,
                help="variable configs: launches rotate over this many copies of the data, so that no launch "
                     "finds its bytes in the 256 MiB Infinity Cache from the one before (memory-side counters "
                     "then see every byte)")
a = ap.parse_args()
lib = _lib.lib
if a.lib:
    lib = ctypes.CDLL(os.path.abspath(a.lib), mode=os.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(lib, name):
            f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
st = torch.cuda.current_stream().cuda_stream
if a.config in ("cfg2", "gen"):
    n, L = a.blocks, a.len
    S, off = (L, 0) if a.config == "cfg2" else (L + 3, 3)
    buf = torch.empty(off + n * S + 64, dtype=torch.uint8, device=dev)
    lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), buf.numel() // 8, 8, 0, 1, 0x5EED0001, None)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ws = torch.empty(max(1, lib.nvl_crc32c_fixed_workspace_bytes(S, L, n)), dtype=torch.uint8, device=dev)
    for _ in range(a.launches):
        assert lib.nvl_crc32c_fixed_dev(buf.data_ptr() + off, S, L, n, None, 0, out.data_ptr(), 0, ws.data_ptr(),
                                        ws.numel(), st) == 0
else:
    if a.config == "cfg3":
        import oracle
        lens = oracle.port().cfg3_lengths(0x5EED0003, 1 << 30).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        total, seed = 1 << 30, 0x5EED0002
    else:
        n = a.blocks
        gap = a.gap if a.config == "varlen" else 4
        if a.config in ("var4097", "varlen"):
            lens = np.full(n, 4097 if a.config == "var4097" else a.len, dtype=np.int64)
        else:
            lens = np.random.default_rng(7).integers(3364, 4110, n).astype(np.int64)
        offs = np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64)
        total, seed = int(offs[-1] + lens[-1]) + 4, 0x5EED0001
    n = lens.size
    if a.shuffle:
        p = np.random.default_rng(1).permutation(n)
        offs, lens = offs[p].copy(), lens[p].copy()
    bufs = [torch.empty(total + 64, dtype=torch.uint8, device=dev) for _ in range(max(1, a.copies))]
    for buf in bufs:
        lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), (total + 64) // 8, 8, 0, 1, seed, None)
    o = torch.from_numpy(offs).to(dev)
    m = torch.from_numpy(lens).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    if a.region:
        wsb = lib.nvl_crc32c_region_workspace_bytes(total, n)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        for it in range(a.launches):
            buf = bufs[it % len(bufs)]
            assert lib.nvl_crc32c_region_dev(buf.data_ptr(), total, o.data_ptr(), m.data_ptr(), None, 0,
                                             out.data_ptr(), n, _lib.FLAG_REGION_SHAPED if a.shaped else 0,
                                             ws.data_ptr(), wsb, st) == 0
        torch.cuda.synchronize()
        print("done region", a.config, hex(int(out[0].item()) & 0xFFFFFFFF))
        sys.exit(0)
    ws = torch.empty(lib.nvl_crc32c_batch_workspace_bytes(n), dtype=torch.uint8, device=dev)
    for it in range(a.launches):
        buf = bufs[it % len(bufs)]
        assert lib.nvl_crc32c_batch_dev(buf.data_ptr(), o.data_ptr(), m.data_ptr(), None, 0, out.data_ptr(), n, 0,
                                        ws.data_ptr(), ws.numel(), st) == 0
torch.cuda.synchronize()
print("done", a.config, hex(int(out[0].item()) & 0xFFFFFFFF))
