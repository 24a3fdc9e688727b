"""Which buffers a pool variant (tools/diag/pool_balance.patch applied to the
in-tree library) leaves unwritten against build/libnvl_crc32c_base.so (the
shipped kernel), config 2, three calls on one workspace; the pool counters
after each call.  (Found the slot-initialisation race of that patch's first
form: the LDS slots were written before the image fill's stores had landed.)"""
import ctypes, os, sys, json
import numpy as np, torch
sys.path.insert(0, os.getcwd())
from nvlevelz_amd import _lib
def load(path):
    lib = ctypes.CDLL(os.path.abspath(path), mode=os.RTLD_LOCAL)
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(lib, name); f.restype = res; f.argtypes = args
    return lib
dev = torch.device("cuda:0"); torch.cuda.set_device(dev)
base = load("build/libnvl_crc32c_base.so"); pool = load("nvlevelz_amd/libnvl_crc32c.so")
for l in (base, pool): assert l.nvl_crc32c_init(0) == 0
n, L = 100000, 4096
buf = torch.empty(n * L, dtype=torch.uint8, device=dev)
base.nvl_crc32c_fill_splitmix(buf.data_ptr(), n, L, 0, 1, 0x5EED0001, None)
st = torch.cuda.current_stream().cuda_stream
ref = torch.zeros(n, dtype=torch.int32, device=dev)
assert base.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, ref.data_ptr(), 0, None, 0, st) == 0
wsb = pool.nvl_crc32c_fixed_workspace_bytes(L, L, n)
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
for it in range(3):
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    assert pool.nvl_crc32c_fixed_dev(buf.data_ptr(), L, L, n, None, 0, out.data_ptr(), 0, ws.data_ptr(), wsb, st) == 0
    torch.cuda.synchronize()
    bad = np.nonzero((out != ref).cpu().numpy())[0]
    nst = n - 312 * 32
    print(json.dumps({"it": it, "wsb": wsb, "nbad": int(bad.size), "first": bad[:10].tolist(),
                      "in_pool": int((bad >= nst).sum()),
                      "blocks_bad": sorted(set(((bad[bad >= nst] - nst) // 32).tolist()))[:40],
                      "within_block_pos": sorted(set(((bad[bad >= nst] - nst) % 32).tolist()))[:40],
                      "ctrs": ws.view(torch.int32).cpu().numpy()[::1024][:8].tolist()}))
