#!/bin/bash
# One GPU call of round-2 work: parity tests, the default bench line, the
# self-spawned 2-rank cfg5 rehearsal (gloo, ranks sharing one GPU), and a
# rocprofv3 kernel trace of the whole-table verify shim bench.
#   bash tools/gpu_round.sh TAG [steps...]    steps: tests bench spawn shims (default: all)
set -o pipefail
TAG=${1:-r02}
shift
STEPS=${*:-tests bench spawn shims}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
run() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "[gpu_round] $(date +%T) $name"
  timeout -k 10 $t "$@" > $OUT/${name}_$TAG.log 2>&1
  local rc=$?
  echo "[gpu_round] $name rc=$rc"
  tail -4 $OUT/${name}_$TAG.log
  [ $rc -eq 0 ] || exit $rc
}
for s in $STEPS; do
  case $s in
    tests) run pytest 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ;;
    bench) run bench 400 python bench.py ;;
    spawn) NVL_BENCH_BACKEND=gloo run spawn 400 python bench.py --gpus 2 --config cfg5 --steps 20 --warmup 3 ;;
    cfg5) run cfg5 400 python bench.py --config cfg5 --steps 50 --warmup 5 --no-cpu --no-e2e ;;
    shims)
      cd /tmp && export TMPDIR=/tmp
      run shims 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shims_$TAG -o run -- \
        python3 $R/bench.py --shims --no-cpu --no-e2e --steps 20 --warmup 5
      cd $R ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
        python3 $R/bench.py --no-cpu --no-e2e --steps 100 --warmup 20
      cd $R ;;
  esac
done
echo "[gpu_round] done"
