set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_rv -o run -- python3 $R/tools/bench_configs.py --configs r,v --reps 20 || exit 1
cd $R && CFG=r timeout -k 10 100 python3 tools/diag/tl.py
