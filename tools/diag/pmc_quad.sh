#!/bin/bash
# Traffic attribution on the region kernel: the quick PMC
# passes over `r` (rand, one-launch region) for the fold without its 16-byte
# quad re-reads (tools/diag/abl_quad.sh `noquad`, wrong results) and the same
# source unedited (`base`).  Build first: bash tools/diag/abl_quad.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PMC_SET=quick NVL_CRC32C_SELFTEST_REPORT_ONLY=1
for v in base noquad; do
  bash tools/pmc.sh q_$v --lib $R/build/libnvl_crc32c_$v.so --config rand --region --shaped --launches 10 \
    > gpurun_out/pmc_q_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pmc_q_$v.log; exit 1; }
  echo "pmc $v ok"
done
O=gpurun_out
python3 tools/pmc_workloads.py $O/r05_pmc_quad.json \
  region_rand_base=$O/pmc_q_base:375720162:crc32c_region_kernel \
  region_rand_noquad=$O/pmc_q_noquad:375720162:crc32c_region_kernel > /dev/null && echo "summary ok"
