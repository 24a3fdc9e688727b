#!/bin/bash
# Counter calibration: tools/diag/pmc_calib (known byte
# counts per access width) and the routed shuffled config-3 workload, each
# pass its own rocprofv3 --pmc run (kernel trace only), raw per-dispatch
# values summarised by tools/diag/pmc_calib_summary.py.
#   bash tools/diag/pmc_calib.sh TAG
set -o pipefail
TAG=${1:-calib}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_calib_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "TCP_TCC_READ_REQ_sum SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/micro -o pass$i -- $R/tools/diag/pmc_calib \
    > $OUT/micro_pass$i.log 2>&1 || { echo "micro pass $i failed: $grp"; tail -5 $OUT/micro_pass$i.log; exit 1; }
  echo "micro pass $i ok: $grp"
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/cfg3s -o pass$i -- python3 $R/tools/prof_workload.py \
    --config cfg3 --shuffle --launches 6 > $OUT/cfg3s_pass$i.log 2>&1 || { echo "cfg3s pass $i failed: $grp"; tail -5 $OUT/cfg3s_pass$i.log; exit 1; }
  echo "cfg3s pass $i ok: $grp"
done
python3 $R/tools/diag/pmc_calib_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
