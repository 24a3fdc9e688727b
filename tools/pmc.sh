#!/bin/bash
# rocprofv3 counter passes (one --pmc group per run, kernel-trace only; never
# combined with sys/runtime traces) over tools/prof_workload.py.
# Usage: bash tools/pmc.sh TAG [workload args...]      (PMC_SET=quick: traffic passes only)
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT -o pass$i -- python3 $R/tools/prof_workload.py "$@" > $OUT/pass$i.log 2>&1 || { echo "pass $i failed: $grp"; tail -5 $OUT/pass$i.log; exit 1; }
  echo "pass $i ok: $grp"
done < <(if [ "${PMC_SET:-full}" = quick ]; then printf '%s\n' "FETCH_SIZE SQ_WAVES" "WRITE_SIZE SQ_WAVES" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum SQ_WAVES"; else cat <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_LOAD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_INST_CYCLES_VMEM_RD
FETCH_SIZE SQ_WAVES
WRITE_SIZE SQ_WAVES
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum SQ_WAVES
GROUPS
fi)
echo "all passes ok"
