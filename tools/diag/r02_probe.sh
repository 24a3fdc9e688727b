set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 120 ./tools/diag/ldpat > $OUT/ldpat.jsonl 2>&1 && cat $OUT/ldpat.jsonl &&
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench_r02b.json 2>$OUT/bench_r02b.err && cat $OUT/bench_r02b.json &&
PMC_SET=quick timeout -k 10 300 bash tools/pmc.sh cfg3_r02 --config cfg3 --launches 10 &&
PMC_SET=quick timeout -k 10 300 bash tools/pmc.sh var4097_r02 --config var4097 --launches 10 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_cfg3_r02 -o run -- python3 $R/tools/prof_workload.py --config cfg3 --launches 20 > $OUT/prof_cfg3.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_var4097_r02 -o run -- python3 $R/tools/prof_workload.py --config var4097 --launches 20 > $OUT/prof_var4097.log 2>&1 &&
cut -d, -f1-4 $OUT/prof_cfg3_r02/run_kernel_stats.csv | cut -c1-120 && cut -d, -f1-4 $OUT/prof_var4097_r02/run_kernel_stats.csv | cut -c1-120
