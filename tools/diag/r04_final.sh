#!/bin/bash
# Round-4 closing evidence on one GPU box (every step time-limited, chained):
# the GPU suite, the configs table and region traces (r04_measure.sh), the
# bench line and its rocprof kernel stats, smoke.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 420 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $O/r04_gpu_tests_final.log 2>&1 || { tail -20 $O/r04_gpu_tests_final.log; exit 1; }
echo "tests ok"
bash $R/tools/diag/r04_measure.sh configs prof || exit 1
timeout -k 10 300 python3 $R/bench.py > $O/r04_bench_final.json 2> $O/r04_bench_final.err || exit 1
echo "bench ok"
(cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profb_final -o run \
  -- python3 $R/bench.py > $O/r04_bench_prof.json 2> $O/r04_bench_prof.err) || exit 1
echo "bench prof ok"
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04_smoke_final.log 2>&1 || exit 1
echo "smoke ok"
