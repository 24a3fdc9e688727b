#!/bin/bash
# One rocprofv3 --pmc pass of instruction counters per workload (kernel-trace
# only, never combined with other traces):  bash tools/diag/pmc_insts.sh TAG
set -o pipefail
TAG=${1:-x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmci_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {  # name, workload args...
  local name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
    SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/$name -o p -- \
    python3 $R/tools/prof_workload.py "$@" --launches 10 > $OUT/$name.log 2>&1 || { echo "pmc $name failed"; tail -3 $OUT/$name.log; exit 1; }
  echo "== $name"; python3 $R/tools/pmc_summary.py $OUT/$name ${KPAT:-crc32c}
}
run cfg2 --config cfg2
KPAT=region_kernel run v_region --config var4097 --region
KPAT=region_kernel run cfg3_region --config cfg3 --region
KPAT=region_fold run v_fold --config var4097 --region
