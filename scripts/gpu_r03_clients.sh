#!/bin/bash
# 120-shard (one rank's share at 8 GPUs) Count q/s vs request-thread count and
# native planner threads.
set -o pipefail
mkdir -p gpurun_out/r03_clients /tmp/pb
for c in ${CLIENTS:-3 6}; do
  for pt in ${PTS:-1 4}; do
    PILOSA_PLAN_THREADS=$pt timeout -k 10 200 python -u bench.py --cols 125000000 --steps 40 --warmup 5 --topn-batches 0 \
      --configs none --data-dir /tmp/pb --clients $c > gpurun_out/r03_clients/c${c}_pt${pt}.log 2>&1 || { tail -c 2000 gpurun_out/r03_clients/c${c}_pt${pt}.log; exit 1; }
    echo "clients=$c plan_threads=$pt $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03_clients/c${c}_pt${pt}.log) $(grep -o '"value": [0-9.]*' gpurun_out/r03_clients/c${c}_pt${pt}.log)"
  done
done
