#!/bin/bash
# Rehearse bench.py's N-rank path (torch.distributed.run, barrier, max-over-ranks
# timing, round-robin shards) on a 1-GPU box: ranks share the GPU and meet over
# gloo (NVL_BENCH_BACKEND=gloo); the 8-GPU node run uses RCCL, one GPU per rank.
# Every line carries the cfg5 object (BASELINE config 5: 10^7 blocks round-robin
# over the N ranks, every rank's digest verified) beside the cfg2 headline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
export NVL_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 50 --warmup 10 --no-cpu > $OUT/dist_n2.json 2> $OUT/dist_n2.err
rc=$?; echo "[dist] n2 rc=$rc"; cat $OUT/dist_n2.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 4 --steps 50 --warmup 10 --no-cpu > $OUT/dist_n4.json 2> $OUT/dist_n4.err
rc=$?; echo "[dist] n4 (self-spawned ranks) rc=$rc"; cat $OUT/dist_n4.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 --steps 50 --warmup 10 --no-cpu > $OUT/dist_n8.json 2> $OUT/dist_n8.err
rc=$?; echo "[dist] n8 rc=$rc"; cat $OUT/dist_n8.json
[ $rc -eq 0 ] || exit $rc
exit 0
