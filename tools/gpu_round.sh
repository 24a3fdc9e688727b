#!/bin/bash
# One GPU call of round work, every step under its own time limit, stopping
# at the first failure.
#   bash tools/gpu_round.sh TAG [steps...]
# steps:
#   tests   pytest -m gpu (parity)
#   bench   the driver's exact command: python3 bench.py --gpus 1 --steps 20 --warmup 5
#   prof    rocprofv3 --kernel-trace --stats of that same command (summary split by phase)
#   spawn   self-spawned 2-rank rehearsals without torchrun (gloo, ranks sharing one GPU):
#           cfg5 (full 10^7-block digest through shard.gather_crcs) and cfg2
#   configs tools/bench_configs.py over 2,3,3R,3S,4,v,vR,vS,r,rR,rS,g,u,uR,uo,big1
#   shims   rocprofv3 kernel trace of the whole-table verify shim bench
#   smoke   __graft_entry__.smoke();  default  python3 bench.py with no flags (the driver's BENCH line)
#   pmc     tools/pmc.sh (full counter set) on cfg2, rand (3364..4109 B), var4097, cfg3
#   ceiling tools/diag/hbm_ceiling (read-only streaming kernels: the measured HBM read ceiling;
#           built here first: hipcc -O3 --offload-arch=gfx950 tools/diag/hbm_ceiling.hip -o tools/diag/hbm_ceiling)
set -o pipefail
TAG=${1:-r03}
shift
STEPS=${*:-tests bench prof spawn configs}
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
    tests) run pytest 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ;;
    bench) run bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    bench100) run bench100 300 python3 bench.py --gpus 1 --steps 300 --warmup 100 --no-cpu --no-e2e ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o run -- \
        python3 $R/bench.py --gpus 1 --steps 20 --warmup 5
      cd $R
      tr=$(ls $OUT/prof_$TAG/*/run_kernel_trace.csv $OUT/prof_$TAG/run_kernel_trace.csv 2>/dev/null | head -1)
      python3 tools/rocprof_summary.py "$tr" $OUT/prof_summary_$TAG.json 20 5 $OUT/prof_timed_stats_$TAG.csv ;;
    spawn)
      NVL_BENCH_BACKEND=gloo run spawn_cfg5 400 python3 bench.py --gpus 2 --config cfg5 --steps 10 --warmup 2 --no-cpu --no-e2e
      NVL_BENCH_BACKEND=gloo run spawn_cfg2 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-e2e ;;
    configs) run configs 600 python3 tools/bench_configs.py --configs 2,3,3R,3S,4,v,vR,vS,r,rR,rS,g,u,uR,uo,big1 ;;
    smoke) run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
    ceiling) run ceiling 120 ./tools/diag/hbm_ceiling ;;
    default) run bench_default 400 python3 bench.py ;;
    pmc)
      for c in cfg2 rand var4097 cfg3; do
        run pmc_$c 400 bash tools/pmc.sh ${TAG}_$c --config $c --launches 10
      done ;;
    shims)
      cd /tmp && export TMPDIR=/tmp
      run shims 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_shims_$TAG -o run -- \
        python3 $R/bench.py --shims --no-cpu --no-e2e --steps 20 --warmup 5
      cd $R ;;
  esac
done
echo "[gpu_round] done"
