#!/bin/bash
# GPU parity, then configs 2-4 timed for the in-tree lib and each variant .so
# given as arguments, alternating (A B A B).  Usage: bash tools/diag/ab_cfgs.sh build/libnvl_crc32c_X.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for round in 1 2; do
  for L in nvlevelz_amd/libnvl_crc32c.so "$@"; do
    echo "== $L"
    timeout -k 10 200 python3 tools/bench_configs.py --lib $L --configs ${AB_CONFIGS:-2,3,4} || exit 1
  done
done
