#!/bin/bash
# Per-kernel times of each workload of tools/prof_workload.py: one rocprofv3
# kernel trace per config, the stats summary copied to gpurun_out/profc_TAG_CFG.csv.
#   bash tools/diag/prof_configs.sh TAG [configs...]   (default: cfg3 var4097 gen rand cfg2)
set -o pipefail
TAG=${1:-x}; shift
CFGS=${*:-cfg3 var4097 gen rand cfg2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc_${TAG}_$c -o run -- \
    python3 $R/tools/prof_workload.py --config $c --launches 20 > $OUT/profc_${TAG}_$c.log 2>&1 || exit 1
  f=$OUT/profc_${TAG}_$c/run_kernel_stats.csv
  cp $f $OUT/profc_${TAG}_$c.csv
  echo "== $c"; cut -d, -f1-8 $f | sed 's/"//g' | head -12
done
