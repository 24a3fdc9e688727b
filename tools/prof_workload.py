"""Fixed workload for rocprofv3 counter passes: config-2 fast path, K launches.
    python3 tools/prof_workload.py [--lib build/libnvl_crc32c_X.so] [--blocks N] [--launches K]"""
import argparse, ctypes, os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from nvlevelz_amd import _lib
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None); ap.add_argument("--blocks", type=int, default=100000)
ap.add_argument("--launches", type=int, default=20); ap.add_argument("--len", type=int, default=4096)
a = ap.parse_args()
lib = _lib.lib
if a.lib:
    lib = ctypes.CDLL(os.path.abspath(a.lib), mode=os.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name); f.restype = res; f.argtypes = args
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
assert lib.nvl_crc32c_init(0) == 0
n, L = a.blocks, a.len
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
lib.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
out = torch.empty(n, dtype=torch.int32, device=dev)
ws = torch.empty(max(1, lib.nvl_crc32c_fixed_workspace_bytes(L, L, n)), dtype=torch.uint8, device=dev)
for _ in range(a.launches):
    assert lib.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, ws.data_ptr(),
                                    ws.numel(), torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
print("done", hex(int(out[0].item()) & 0xFFFFFFFF))
