#!/bin/bash
# Kernel-trace breakdown of the config-3 (variable-length) pipeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cfg3 -o run -- python3 $R/tools/bench_configs.py --configs 3 ${PROF_LIB:+--lib $PROF_LIB} > $R/gpurun_out/prof_cfg3.log 2>&1
python3 - <<'PY'
import csv, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
rows = list(csv.DictReader(open(f"{R}/gpurun_out/prof_cfg3/run_kernel_stats.csv")))
for r in rows:
    print(f'{float(r["AverageNs"])/1000:10.1f} us  x{r["Calls"]:>4}  {r["Name"][:90]}')
PY
