#!/bin/bash
# Ablations of the region kernel (wrong results; tools/diag/ab_region.py times them):
#   rnoev    no event work: no buffer event is looked for or recorded (windows and cursors stay)
#   rnowin   rnoev without the metadata windows (no window loads, no cursor search)
#   rpure    rnowin without the in-launch fold (the owned-buffer loop stores 0): the chunk pass alone
# (the fold's own ablations: tools/diag/abl_tail.sh)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
python3 - "$SRC" "$R/build" <<'PY'
import sys
src, out = sys.argv[1], sys.argv[2]
s = open(src).read()
def sub(t, a, b, n=1):
    assert t.count(a) >= n, a
    return t.replace(a, b)
noev = sub(s, "const bool any_ev = !halo && __ballot(le.sv || le.ev) != 0u;", "const bool any_ev = false;")
noev = sub(noev, "} else if (any_ev || (cursor + 64u < g.n && lane_u64(w.s, 63) < (ca + cu) * kChunk)) {",
           "} else if (false) {")
open(out + "/abl_rnoev.hip", "w").write(noev)
nowin = sub(noev, "    const WinRaw nwr = load_win(g, ncur, lane);", "    const WinRaw nwr = WinRaw{0u, 0u};")
nowin = sub(nowin, "  uint64_t cursor = cu ? region_search(g, ca * kChunk, lane, probe) : g.n;", "  uint64_t cursor = 0u;")
open(out + "/abl_rnowin.hip", "w").write(nowin)
a = nowin.index("  const uint64_t nsl = ")
b = nowin.index("__global__ __launch_bounds__(kThreads, 1) void crc32c_region_kernel")
pure = nowin[:a] + ("  __syncthreads();\n  for (uint64_t i = ib + threadIdx.x; i < ib1; i += kThreads) ka.out[i] = (uint32_t)c0w;\n"
                    "}\n\n") + nowin[b:]
open(out + "/abl_rpure.hip", "w").write(pure)
PY
for v in rnoev rnowin rpure; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null 2>&1
done
echo built build/libnvl_crc32c_{rnoev,rnowin,rpure}.so
