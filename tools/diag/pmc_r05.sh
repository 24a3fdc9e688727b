#!/bin/bash
# Round-5 PMC evidence: quick counter passes (traffic by request size,
# FETCH/WRITE_SIZE, instruction counts) per workload, then one summary.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export PMC_SET=quick
run() { bash tools/pmc.sh "$@" > gpurun_out/pmc_$1.log 2>&1 || { echo "pmc $1 failed"; tail -5 gpurun_out/pmc_$1.log; exit 1; }; echo "pmc $1 ok"; }
run r05_cfg2 --config cfg2 --launches 10
run r05_rS --config rand --region --shaped --launches 10
run r05_vS --config var4097 --region --shaped --launches 10
run r05_3S --config cfg3 --region --shaped --launches 10
run r05_r --config rand --launches 10
run r05_ru --config rand --shuffle --launches 10
run r05_3u --config cfg3 --shuffle --launches 10
run r05_3uc --config cfg3 --shuffle --copies 2 --launches 10
run r05_ruc --config rand --shuffle --copies 2 --launches 10
run r05_rSc --config rand --region --shaped --copies 2 --launches 10
O=gpurun_out
python3 tools/pmc_workloads.py $O/r05_pmc_summary.json \
  cfg2=$O/pmc_r05_cfg2:410000000:crc32c_fixed_kernel \
  region_rand=$O/pmc_r05_rS:375720162:crc32c_region_kernel \
  region_var4097=$O/pmc_r05_vS:411700000:crc32c_region_kernel \
  region_cfg3=$O/pmc_r05_3S:1074133888:crc32c_region_kernel \
  routed_rand=$O/pmc_r05_r:375720162:crc32c_route_plan,crc32c_route_kernel,crc32c_var_fused_kernel \
  routed_rand_shuffled=$O/pmc_r05_ru:375720162:crc32c_route_plan,crc32c_route_kernel,crc32c_var_fused_kernel \
  routed_cfg3_shuffled=$O/pmc_r05_3u:1074133888:crc32c_route_plan,crc32c_route_kernel,crc32c_var_fused_kernel \
  routed_cfg3_shuffled_2copies=$O/pmc_r05_3uc:1074133888:crc32c_route_plan,crc32c_route_kernel,crc32c_var_fused_kernel \
  routed_rand_shuffled_2copies=$O/pmc_r05_ruc:375720162:crc32c_route_plan,crc32c_route_kernel,crc32c_var_fused_kernel \
  region_rand_2copies=$O/pmc_r05_rSc:375720162:crc32c_region_kernel \
  > /dev/null && echo "summary ok"
