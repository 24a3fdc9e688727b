#!/bin/bash
# One GPU session producing the round's evidence: parity tests, smoke, bench
# (+e2e), rocprofv3 kernel-trace stats of the bench command, PMC traffic passes,
# and the config 2/3/4 timing table.   Usage: bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
echo "[gpu_check] $(date) start tag=$TAG"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "[gpu_check] pytest rc=$rc"; tail -3 $OUT/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
rc=$?; echo "[gpu_check] smoke rc=$rc"; tail -1 $OUT/smoke_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "[gpu_check] bench rc=$rc"; cat $OUT/bench_$TAG.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bench_configs.py > $OUT/configs_$TAG.jsonl 2> $OUT/configs_$TAG.err
rc=$?; echo "[gpu_check] configs rc=$rc"; cat $OUT/configs_$TAG.jsonl
[ $rc -eq 0 ] || exit $rc
PMC_SET=quick bash tools/pmc.sh $TAG --launches 10 > $OUT/pmc_$TAG.log 2>&1
rc=$?; echo "[gpu_check] pmc rc=$rc"; tail -1 $OUT/pmc_$TAG.log
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python3 $R/bench.py --no-cpu --steps 50 --warmup 5 > $OUT/prof_$TAG.log 2>&1
rc=$?; echo "[gpu_check] rocprof rc=$rc"
exit $rc
