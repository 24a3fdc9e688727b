#!/bin/bash
# Per-kernel mean durations (rocprofv3 --kernel-trace --stats) of kernel
# variants on prof_workload.py configs.
#   bash tools/diag/prof_variants.sh "main nocomp" "var4097 gen varlen,--len,4096,--gap,3"
# (a config with commas passes the rest as prof_workload.py arguments)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export NVL_CRC32C_SELFTEST_REPORT_ONLY=1
for v in $1; do
  lib=""; [ "$v" = main ] || lib="--lib $R/build/libnvl_crc32c_$v.so"
  for c in $2; do
    tag=$(echo $c | tr -c 'A-Za-z0-9\n' '_')
    d=$OUT/pv_${v}_$tag
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 $R/tools/prof_workload.py --config ${c//,/ } --launches 20 $lib > $d.log 2>&1 || exit 1
    python3 - $d/run_kernel_stats.csv $v $c <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if int(r["Calls"]) >= 20]
print(sys.argv[2], sys.argv[3], " | ".join(f'{r["Name"].split("(")[0].split("::")[-1][:28]} {float(r["AverageNs"])/1e3:.1f}' for r in rows))
PY
  done
done
