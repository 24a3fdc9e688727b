#!/bin/bash
# Kernel trace of the region path (nvl_crc32c_region_dev) per workload:
#   bash tools/diag/prof_region.sh TAG [configs...]   (default: cfg3 var4097 rand)
set -o pipefail
TAG=${1:-x}; shift
CFGS=${*:-cfg3 var4097 rand}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profr_${TAG}_$c -o run -- \
    python3 $R/tools/prof_workload.py --config $c --launches 20 --region > $OUT/profr_${TAG}_$c.log 2>&1 || exit 1
  f=$OUT/profr_${TAG}_$c/run_kernel_stats.csv
  cp $f $OUT/profr_${TAG}_$c.csv
  echo "== $c"; cut -d, -f1-8 $f | sed 's/"//g' | head -12
done
