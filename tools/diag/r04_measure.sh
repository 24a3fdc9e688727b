#!/bin/bash
# Round-4 measurement pass on one GPU box (every step time-limited, chained):
#   configs table, region kernel traces, shim latency, isolated cfg2 launch
#   split, PMC traffic of the region and head/fused kernels.
#   bash tools/diag/r04_measure.sh [steps...]   (default: all)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
STEPS=${*:-configs prof shims iso pmc}
for s in $STEPS; do
  case $s in
    configs)
      timeout -k 10 400 python3 $R/tools/bench_configs.py --configs 2,3R,vR,rR,4,big1,3,v,r --reps 30 \
        > $O/r04_configs.jsonl 2> $O/r04_configs.err || exit 1 ;;
    prof)
      (cd /tmp && TMPDIR=/tmp bash $R/tools/diag/prof_region.sh r04 cfg3 var4097 rand > $O/r04_prof_region.log 2>&1) || exit 1 ;;
    shims)
      timeout -k 10 500 python3 $R/tools/shim_latency.py --reps 15 --out $O/r04_shim_latency.jsonl \
        > $O/r04_shim_latency.log 2>&1 || exit 1 ;;
    iso)
      LIB=$R/build/libnvl_crc32c_stamps.so timeout -k 10 200 python3 $R/tools/diag/iso_split.py \
        > $O/r04_iso_split.jsonl 2> $O/r04_iso_split.err || exit 1 ;;
    pmc)
      for w in "region_var4097 --config var4097 --region" "region_cfg3 --config cfg3 --region" \
               "region_rand --config rand --region" "batch_var4097 --config var4097" "batch_cfg3 --config cfg3"; do
        set -- $w; tag=$1; shift
        PMC_SET=quick bash $R/tools/pmc.sh r04_$tag "$@" > $O/pmc_r04_$tag.log 2>&1 || { tail -5 $O/pmc_r04_$tag.log; exit 1; }
      done ;;
  esac
  echo "step $s ok"
done
