#!/bin/bash
# One GPU call of round evidence on the current tree: parity tests, smoke, the
# default bench line, the config table, rocprofv3 kernel stats of the bench
# and of every config workload, PMC traffic passes of the variable-length
# kernels, and the whole-table-verify shim bench under rocprofv3.
#   bash tools/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
step() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "[evidence] $(date +%T) $name"
  timeout -k 10 $t "$@" > $OUT/${name}_$TAG.log 2>&1
  local rc=$?
  echo "[evidence] $name rc=$rc"
  tail -3 $OUT/${name}_$TAG.log
  [ $rc -eq 0 ] || exit $rc
}
step pytest 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py
step configs 400 python tools/bench_configs.py --configs 2,3,4,v,g,r
step profc 600 bash tools/diag/prof_configs.sh $TAG cfg3 var4097 rand gen cfg2
PMC_SET=quick step pmc3 300 bash tools/pmc.sh ${TAG}_cfg3 --config cfg3 --launches 10
PMC_SET=quick step pmcv 300 bash tools/pmc.sh ${TAG}_var4097 --config var4097 --launches 10
cd /tmp && export TMPDIR=/tmp
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
  python3 $R/bench.py --no-cpu --no-e2e --steps 100 --warmup 20
step shims 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shims_$TAG -o run -- \
  python3 $R/bench.py --shims --no-cpu --no-e2e --steps 20 --warmup 5
echo "[evidence] done"
