#!/bin/bash
# A/B of kernel variants (build/libnvl_crc32c_<name>.so, `make variant`) on the
# config table of tools/bench_configs.py; "main" = the in-tree library.
#   bash tools/diag/ab_variants.sh "main r01 w8u1" 2,3,v
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
# variants are -DNVL_DEV_TUNING builds: an ablation with wrong results still runs (the
# shipped library ignores this switch)
export NVL_CRC32C_SELFTEST_REPORT_ONLY=1
for v in $1; do
  lib=""; [ "$v" = main ] || lib="--lib build/libnvl_crc32c_$v.so"
  timeout -k 10 300 python tools/bench_configs.py $lib --configs ${2:-2,3,v} 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || exit 1
done
