#!/bin/bash
# Scheduler A with the grid's buffer pairs interleaved over the workgroups
# (pair p to workgroup p mod G) instead of one contiguous range per
# workgroup: at any moment the chip reads one moving window of the batch,
# as the grid-stride read ceiling does (tools/diag/hbm_ceiling.hip).  Timed
# by tools/ab_bench.py; `base` is the unedited source built the same way.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
python3 - "$SRC" "$R/build" <<'PY'
import sys
src, out = sys.argv[1], sys.argv[2]
s = open(src).read()
a = """  const uint64_t B0 = g.n * blockIdx.x / gridDim.x;
  const uint64_t B1 = g.n * (blockIdx.x + 1) / gridDim.x;
  // The range's last kTail buffers are single-buffer units: a CU's waves
  // then finish within half a unit of each other instead of a whole one.
  const uint32_t cnt = (uint32_t)(B1 - B0);"""
b = """  const uint64_t Gd = gridDim.x, bb = blockIdx.x;
  const uint64_t P = (g.n + 1u) / 2u;
  const uint64_t npb = bb < P ? (P - bb + Gd - 1u) / Gd : 0u;
  const bool odd_last = (g.n & 1u) && npb && ((P - 1u) % Gd == bb);
  const uint32_t cnt = (uint32_t)(2u * npb - (odd_last ? 1u : 0u));
  auto gidx = [&](uint64_t j) -> uint64_t { return 2u * ((j >> 1) * Gd + bb) + (j & 1u); };"""
c = """    const uint64_t i = u < nfull ? B0 + (uint64_t)u * U + (uint64_t)k : B0 + (uint64_t)nfull * U + (u - nfull);"""
d = """    const uint64_t i = gidx(u < nfull ? (uint64_t)u * U + (uint64_t)k : (uint64_t)nfull * U + (u - nfull));"""
assert s.count(a) == 1 and s.count(c) == 1
open(out + "/abl_interleave.hip", "w").write(s.replace(a, b).replace(c, d))
open(out + "/abl_base.hip", "w").write(s)
PY
for v in interleave base; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null &
done
wait
ls $R/build/libnvl_crc32c_{interleave,base}.so
