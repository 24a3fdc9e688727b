#!/bin/bash
# Plan-kernel shapes (timed by tools/diag/ab_region.py with AB_FLAGS=0 -- the
# checked region_dev call): threads per workgroup x pairs per thread x the
# most workgroups.  t1024p4m64 is the shipped shape.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
VARS="t1024p4m64 t256p4m128 t512p2m128 t1024p1m128 t256p2m256 t256p1m256"
python3 - "$SRC" "$R/build" $VARS <<'PY'
import re, sys
src, out, names = sys.argv[1], sys.argv[2], sys.argv[3:]
s = open(src).read()
a = "constexpr uint32_t kPlanT = 1024, kPlanPer = 4;"
b = "constexpr uint32_t kRoutePlanMax = 64;"
assert s.count(a) == 1 and s.count(b) == 1
for name in names:
    t, p, m = map(int, re.match(r"t(\d+)p(\d+)m(\d+)", name).groups())
    open(out + "/abl_%s.hip" % name, "w").write(
        s.replace(a, "constexpr uint32_t kPlanT = %d, kPlanPer = %d;" % (t, p)).replace(b, "constexpr uint32_t kRoutePlanMax = %d;" % m))
PY
for v in $VARS; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null &
done
wait
for v in $VARS; do ls $R/build/libnvl_crc32c_$v.so; done
