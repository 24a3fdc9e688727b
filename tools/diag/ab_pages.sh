set -o pipefail
export NVL_CRC32C_SELFTEST_REPORT_ONLY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_route.py tests/test_gpu_route_fuzz.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pages.log 2>&1 || { tail -30 gpurun_out/t_pages.log; exit 1; }
tail -2 gpurun_out/t_pages.log
for c in uR uoR rR vR 3R; do
  AB_FLAGS=0 timeout -k 10 200 python -u tools/diag/ab_region.py $c build/libnvl_crc32c_head.so build/libnvl_crc32c_pages.so > gpurun_out/ab_pages_$c.jsonl 2>&1 || { tail -5 gpurun_out/ab_pages_$c.jsonl; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/ab_pages_$c.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d.get('config'), d.get('variant'), d['period_us'], d.get('single_median_us'), d.get('same_as_first'))
"
done
