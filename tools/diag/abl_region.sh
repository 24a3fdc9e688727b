#!/bin/bash
# Ablations of the region path (wrong results; tools/diag/ab_region.py times them):
#   rnoev    no event work: every unit takes chains_keep, region_events never runs
#            (the window loads and cursors stay)
#   rnowin   rnoev without the metadata windows (no window loads, no cursor)
#   rnofold  the full chunk kernel, no fold kernel launch
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
sed -e 's|^    const bool any_ev = __ballot(le.sv \|\| le.ev) != 0u;|    const bool any_ev = false;|' \
    -e 's|^    if (any_ev \|\| (cursor + 64u < g.n \&\& lane_u64(w.s, 63) < (ca + cu) \* kChunk))|    if (false)|' \
    $SRC > $R/build/abl_rnoev.hip
[ $(grep -c 'const bool any_ev = false;\|    if (false)$' $R/build/abl_rnoev.hip) -eq 2 ] || { echo "rnoev: anchors" >&2; exit 1; }
sed -e 's|^    const WinRaw nwr = load_win(g, ncur, lane);|    const WinRaw nwr = WinRaw{0u, 0u};|' \
    -e 's|^  uint64_t cursor = cu ? region_search(g, ca \* kChunk, lane) : g.n;|  uint64_t cursor = 0u;|' \
    $R/build/abl_rnoev.hip > $R/build/abl_rnowin.hip
[ $(grep -c 'WinRaw nwr = WinRaw{0u, 0u};\|uint64_t cursor = 0u;' $R/build/abl_rnowin.hip) -eq 2 ] || { echo "rnowin: anchors" >&2; exit 1; }
sed -e 's|^  dev::RegionFold f{|  return hipGetLastError();\n  dev::RegionFold f{|' $SRC > $R/build/abl_rnofold.hip
[ $(grep -c '^  return hipGetLastError();$' $R/build/abl_rnofold.hip) -ge 1 ] || { echo "rnofold: anchors" >&2; exit 1; }
for v in rnoev rnowin rnofold; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{rnoev,rnowin,rnofold}.so
