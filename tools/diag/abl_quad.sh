#!/bin/bash
# Ablation of the region fold's 16-byte quad re-reads (wrong results; timed by
# tools/diag/ab_region.py): `noquad` -- fold_in loads no quads (zeros), i.e.
# what carrying the piece words in the event records would save at most;
# `base` -- the same source unedited, built the same way.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
python3 - "$SRC" "$R/build" <<'PY'
import sys
src, out = sys.argv[1], sys.argv[2]
s = open(src).read()
a = "  f.vs = ld16c((uintptr_t)g.grid + (s & ~(uint64_t)15));"
b = "  f.ve = ld16c((uintptr_t)g.grid + (oe == kChunk ? e - 16u : (e & ~(uint64_t)15)));"
assert a in s and b in s
open(out + "/abl_noquad.hip", "w").write(s.replace(a, "  f.vs = u32x4{0u, 0u, 0u, 0u};").replace(b, "  f.ve = u32x4{(uint32_t)s, 0u, 0u, 0u};"))
open(out + "/abl_base.hip", "w").write(s)
PY
for v in noquad base; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{noquad,base}.so
