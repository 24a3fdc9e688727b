#!/bin/bash
# Where a routed call's overhead goes (timed by tools/diag/ab_region.py with
# AB_FLAGS=0, i.e. the checked region_dev call; a region-shaped batch, every
# call the same batch and workspace, so the plan's partials of an earlier call
# stand in for a skipped plan): `noplan` -- launch_routed skips the plan
# launch; `nofused` -- it skips the body kernel (its early exit); `bare` --
# both: the route kernel alone; `base` -- unedited, built the same way.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
python3 - "$SRC" "$R/build" <<'PY'
import sys
src, out = sys.argv[1], sys.argv[2]
s = open(src).read()
plan = "  if (lc.ev_start)\n    hipExtLaunchKernelGGL(dev::crc32c_route_plan,"
fused = "  if (lc.ev_stop)\n    hipExtLaunchKernelGGL(dev::crc32c_var_fused_kernel,"
assert s.count(plan) == 1 and s.count(fused) == 1
np_ = s.replace(plan, "  if (false) {} else if (lc.ev_start)\n    hipExtLaunchKernelGGL(dev::crc32c_route_plan,")
np_ = np_.replace("  else\n    hipLaunchKernelGGL(dev::crc32c_route_plan,", "  else if (false)\n    hipLaunchKernelGGL(dev::crc32c_route_plan,")
assert np_ != s
nf = s.replace(fused, "  if (true) return hipSuccess;\n" + fused)
bare = np_.replace(fused, "  if (true) return hipSuccess;\n" + fused)
for name, text in (("noplan", np_), ("nofused", nf), ("bare", bare), ("base", s)):
    open(out + "/abl_%s.hip" % name, "w").write(text)
PY
for v in noplan nofused bare base; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{noplan,nofused,bare,base}.so
