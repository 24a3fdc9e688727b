#!/bin/bash
# Ablations of the region kernel's in-launch fold (wrong results; tools/diag/ab_region.py times them):
#   tnop   the owned-buffer loop stores 0 (barrier, halo and ownership searches only)
#   tload  the loop loads metadata and records and stores their XOR (no fold arithmetic)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
python3 - "$SRC" "$R/build" <<'PY'
import sys
src, out = sys.argv[1], sys.argv[2]
s = open(src).read()
a = s.index("  const uint64_t nsl = ")
b = s.index("__global__ __launch_bounds__(kThreads, 1) void crc32c_region_kernel")
body = s[a:b]
nop = "  __syncthreads();\n  for (uint64_t i = ib + threadIdx.x; i < ib1; i += kThreads) ka.out[i] = (uint32_t)c0w;\n}\n\n"
load = ("  __syncthreads();\n  for (uint64_t i = ib + threadIdx.x; i < ib1; i += kThreads) {\n"
        "    const uint64_t off = ldg64(g.offsets, i), L = ldg64(g.lengths, i);\n"
        "    const uint4 q_s = g.qs[i], q_e = g.qe[i];\n"
        "    ka.out[i] = (uint32_t)(off ^ L ^ c0w) ^ q_s.x ^ q_e.x ^ q_s.z ^ q_e.z;\n  }\n}\n\n")
open(out + "/abl_tnop.hip", "w").write(s[:a] + nop + s[b:])
open(out + "/abl_tload.hip", "w").write(s[:a] + load + s[b:])
PY
for v in tnop tload; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{tnop,tload}.so
