#!/bin/bash
# Ablations of the variable-length passes (wrong results, same loads):
#   lo     the short-mode drain (drain_list) and scheduler C (run_bufs) run
#          no chains: each pass XORs its 16 built words into its "raw", so
#          every loaded word is still consumed -- what the loads, the
#          transpose/realign and the scheduling cost without the lookups
#   nofix  the drain's passes skip head_fix (no masking / ~init injection)
# Built from copies of the kernel source under build/; compare with
# tools/diag/ab_variants.sh "main lo nofix" 3,v,r,g.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
XOR='{ for (int q_ = 0; q_ < 2; ++q_) { uint32_t x_ = 0; for (int k_ = 0; k_ < 16; ++k_) x_ ^= w[q_][k_]; RAW[q_] = x_; } }'
sed -e "s|^    chains<2, false>(lds, lb, w, lane, raws);|    ${XOR//RAW/raws}|" \
    -e "s|^      chains<2, false>(lds, lb, w, lane, raws);|      ${XOR//RAW/raws}|" $SRC > $R/build/abl_lo.hip
[ $(grep -c 'x_ ^= w\[q_\]' $R/build/abl_lo.hip) -eq 2 ] || { echo "lo: anchors not found" >&2; exit 1; }
sed -e 's|^    realign_general(A.ce, true, |    realign_general(A.ce, false, |' \
    -e 's|^    realign_general(B.ce, true, |    realign_general(B.ce, false, |' $SRC > $R/build/abl_nofix.hip
[ $(grep -c 'realign_general([AB].ce, false' $R/build/abl_nofix.hip) -eq 2 ] || { echo "nofix: anchors not found" >&2; exit 1; }
for v in lo nofix; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{lo,nofix}.so
# scheduler C (run_bufs) ablations, for config 3's body kernel:
#   noacc  no shift4096 in the per-chunk accumulation nor on the head registers
#   nohv   no hc[i] load per chunk (the head register taken as 0)
sed -e 's|    acc = (first ? ((q.f \& kPosHeadIn) ? hs : 0u) : shift4096(lds, acc, lane)) ^ raw;|    acc = (first ? hs : acc) ^ raw;|' \
    -e 's|    const uint32_t hs0 = shift4096(lds, hv0, lane), hs1 = shift4096(lds, hv1, lane);|    const uint32_t hs0 = hv0, hs1 = hv1;|' $SRC > $R/build/abl_noacc.hip
[ $(grep -c 'acc = (first ? hs : acc) ^ raw;\|const uint32_t hs0 = hv0, hs1 = hv1;' $R/build/abl_noacc.hip) -eq 2 ] || { echo "noacc: anchors not found" >&2; exit 1; }
sed -e 's|^  hv = __builtin_nontemporal_load((const __attribute__((address_space(1))) uint32_t\*)ha);|  hv = (uint32_t)ha;|' $SRC > $R/build/abl_nohv.hip
[ $(grep -c 'hv = (uint32_t)ha;' $R/build/abl_nohv.hip) -eq 1 ] || { echo "nohv: anchors not found" >&2; exit 1; }
for v in noacc nohv; do
  make -C $R/nvlevelz_amd/csrc variant NAME=$v VSRC=$R/build/abl_$v.hip VFLAGS="-I$R/nvlevelz_amd/csrc" > /dev/null
done
echo built build/libnvl_crc32c_{noacc,nohv}.so
