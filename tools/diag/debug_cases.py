"""Kernel debugging: small fixed/varlen cases vs the oracle with per-case detail."""
import os, sys
os.environ["NVL_CRC32C_SELFTEST_REPORT_ONLY"] = "1"
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
import numpy as np, torch, oracle
from nvlevelz_amd import crc32c as C
p = oracle.port()
dev = torch.device("cuda:0")
C.init(0)
def fixed(host, stride, L, n, init=0):
    b = torch.from_numpy(host).to(dev)
    g = C.to_u32(C.extend_fixed(b, stride, L, n, init))
    w = p.fixed(host, stride, L, n, np.full(n, init, dtype=np.uint32))
    return g, w
cases = []
z = np.zeros(4096, dtype=np.uint8)
cases.append(("zeros4096", z))
o = np.zeros(4096, dtype=np.uint8); o[0] = 1; cases.append(("byte0=1", o))
o = np.zeros(4096, dtype=np.uint8); o[64] = 1; cases.append(("byte64=1", o))
o = np.zeros(4096, dtype=np.uint8); o[4095] = 1; cases.append(("byte4095=1", o))
o = np.zeros(4096, dtype=np.uint8); o[4032] = 1; cases.append(("byte4032=1", o))
o = np.zeros(4096, dtype=np.uint8); o[4033] = 1; cases.append(("byte4033=1", o))
o = np.zeros(4096, dtype=np.uint8); o[4034] = 1; cases.append(("byte4034=1", o))
o = np.zeros(4096, dtype=np.uint8); o[4035] = 1; cases.append(("byte4035=1", o))
o = np.zeros(4096, dtype=np.uint8); o[4036] = 1; cases.append(("byte4036=1", o))
o = np.zeros(4096, dtype=np.uint8); o[3968] = 1; cases.append(("byte3968=1 (lane62)", o))
o = np.zeros(4096, dtype=np.uint8); o[2048] = 1; cases.append(("byte2048=1 (lane32)", o))
cases.append(("random", p.fill(1, 0, 4096)))
for name, h in cases:
    for init in (0, 0xFFFFFFFF):
        g, w = fixed(h, 4096, 4096, 1, init)
        print(f"{name:24s} init={init:08x} gpu={int(g[0]):08x} want={int(w[0]):08x} {'ok' if g[0]==w[0] else 'BAD'}")
h = p.fill(2, 0, 64 * 4096)
g, w = fixed(h, 4096, 4096, 64)
print("64 blocks mismatches:", int((g != w).sum()))
