#!/bin/bash
# Ablation: butterfly / shift4096 lookups WITHOUT bank conflicts.
# Builds build/libnvl_crc32c_noconf.so from a copy of the kernel source whose
# lane_lookup keeps the data byte's top three bits (so every lookup still
# depends on the data) but takes the bank from the lane (lane & 31): the same
# instruction count and dependency chain as the product, conflict-free, wrong
# results.  Its time against the product's (tools/diag/ab_variants.sh
# "main noconf") bounds what removing the combine's bank conflicts can gain.
#   bash tools/diag/abl_comb.sh            (CPU: build)
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p $R/build
SRC=$R/nvlevelz_amd/csrc/crc32c_kernels.hip
DST=$R/build/abl_noconf.hip
sed -e 's|return lds_u32(lds + OFF, base + (b << 2));|return lds_u32(lds + OFF, base + (((b \& 0xE0u) \| (__lane_id() \& 31u)) << 2));|' $SRC > $DST
grep -q '__lane_id() & 31u' $DST || { echo "pattern not found in lane_lookup" >&2; exit 1; }
make -C $R/nvlevelz_amd/csrc variant NAME=noconf VSRC=$DST VFLAGS="-I$R/nvlevelz_amd/csrc"
