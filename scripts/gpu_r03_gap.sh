#!/bin/bash
# 120-shard Count: blocking vs polled result wait, then a kernel trace of the
# polled run for the inter-batch GPU idle.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r03_gap /tmp/pb
A="--cols 125000000 --steps 40 --warmup 5 --topn-batches 0 --configs none --data-dir /tmp/pb --clients 3"
for poll in 0 0.00005 0.0002; do
  PILOSA_D2H_POLL=$poll timeout -k 10 200 python -u bench.py $A > gpurun_out/r03_gap/poll_$poll.log 2>&1 || { tail -c 2000 gpurun_out/r03_gap/poll_$poll.log; exit 1; }
  echo "poll=$poll $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r03_gap/poll_$poll.log) $(grep -o '"value": [0-9.]*' gpurun_out/r03_gap/poll_$poll.log)"
done
cd /tmp && export TMPDIR=/tmp
PILOSA_D2H_POLL=0.00005 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03_gap/prof -o gap -- \
  python3 $R/bench.py $A > $R/gpurun_out/r03_gap/prof.log 2>&1 || { tail -c 2000 $R/gpurun_out/r03_gap/prof.log; exit 1; }
echo traced
