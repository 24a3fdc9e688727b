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
#   rbare    rnowin without the batch check (no metadata reads at all): the bare chunk pass
sed -e 's|^  const uint64_t co = ldg64(g.offsets, ci), cl = ldg64(g.lengths, ci);|  const uint64_t co = 0, cl = 0;|' \
    -e 's|^  const uint64_t po = ldg64(g.offsets, cp), pl = ldg64(g.lengths, cp);|  const uint64_t po = 0, pl = 0;|' \
    -e 's|^    for (uint64_t i = i0 + 64u + (uint64_t)lane; i < i1; i += 64u) {  // slices of more than 64 buffers|    for (uint64_t i = i1; i < i1; i += 64u) {|' \
    $R/build/abl_rnowin.hip > $R/build/abl_rbare.hip
[ $(grep -c 'const uint64_t co = 0, cl = 0;\|const uint64_t po = 0, pl = 0;\|for (uint64_t i = i1; i < i1;' $R/build/abl_rbare.hip) -eq 3 ] || { echo "rbare: anchors" >&2; exit 1; }
#   rpure    rbare without the fold kernel: the chunk pass alone
sed -e 's|^  dev::RegionFold f{|  return hipGetLastError();\n  dev::RegionFold f{|' $R/build/abl_rbare.hip > $R/build/abl_rpure.hip
for v in rnoev rnowin rnofold rbare rpure; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{rnoev,rnowin,rnofold,rbare,rpure}.so
