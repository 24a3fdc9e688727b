#!/bin/bash
# Round-3 probes on the GPU box (after tools/diag/abl_comb.sh and the stamps
# variant were built on the CPU side):
#   combine bank-conflict ablation vs the product on the config table, and the
#   head kernel's phase timeline on r and v.
#   bash tools/diag/r03_probe.sh TAG
set -o pipefail
TAG=${1:-r03}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
run() {  # name timeout cmd...
  local name=$1 t=$2
  shift 2
  echo "[probe] $(date +%T) $name"
  timeout -k 10 $t "$@" > $OUT/${name}_$TAG.log 2>&1
  local rc=$?
  echo "[probe] $name rc=$rc"
  tail -4 $OUT/${name}_$TAG.log
  [ $rc -eq 0 ] || exit $rc
}
run abcomb 500 bash tools/diag/ab_variants.sh "main noconf main noconf" ${CFGS:-2,3,4,v,g,r}
CFG=r LIB=build/libnvl_crc32c_stamps.so run tl_r 120 python3 tools/diag/tl.py
CFG=v LIB=build/libnvl_crc32c_stamps.so run tl_v 120 python3 tools/diag/tl.py
CFG=3 LIB=build/libnvl_crc32c_stamps.so run tl_3 120 python3 tools/diag/tl.py
echo "[probe] done"
