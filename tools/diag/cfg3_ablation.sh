export NVL_CRC32C_SELFTEST_REPORT_ONLY=1
for v in base noreal nomask nocomp; do timeout -k 10 120 python tools/bench_configs.py --configs 3 --lib build/libnvl_crc32c_$v.so 2>&1 | grep -v -e amdgpu.ids -e self-test | sed "s/^/$v /"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg3 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs 3 > /dev/null 2>&1
cut -d, -f1-4 $GRAFT_REPO_ROOT/gpurun_out/prof_cfg3/run_kernel_stats.csv | cut -c1-150
