#!/bin/bash
# rocprofv3 kernel trace of routed calls (v, r through nvl_crc32c_batch_dev)
# beside the single-launch region path (vS, rS), summarised by route_tl.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for c in v vS r rS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_route_$c -o run -- \
    python3 $R/tools/bench_configs.py --configs $c --reps 30 --warm-ms 20 > $R/gpurun_out/prof_route_$c.log 2>&1 || exit 1
  tr=$(ls $R/gpurun_out/prof_route_$c/*/run_kernel_trace.csv $R/gpurun_out/prof_route_$c/run_kernel_trace.csv 2>/dev/null | head -1)
  echo "== $c"; python3 $R/tools/diag/route_tl.py "$tr"
done
