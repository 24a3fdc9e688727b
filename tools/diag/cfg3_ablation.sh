#!/bin/bash
# Config-3 ablations (wrong results by design: self-test reported, not fatal)
# and the kernel-trace breakdown of the current pipeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export NVL_CRC32C_SELFTEST_REPORT_ONLY=1
for v in ${CFG3_VARIANTS:-c3_cur c3_noreal c3_nomask c3_nocomp c3_nofold}; do
  timeout -k 10 120 python tools/bench_configs.py --configs 3 --lib build/libnvl_crc32c_$v.so 2>&1 | grep -v -e amdgpu.ids -e self-test | sed "s/^/$v /" || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cfg3 -o run -- python3 $R/tools/bench_configs.py --configs 3 > /dev/null 2>&1 || exit 1
cut -d, -f1-4 $R/gpurun_out/prof_cfg3/run_kernel_stats.csv | cut -c1-150
