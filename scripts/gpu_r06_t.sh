#!/bin/bash
# Round 6, call T: serving Count with each group-commit thread's batches on a
# HIP stream of its own (PILOSA_HTTP_THREAD_STREAMS=1) vs the shared stream.
set -o pipefail
O=gpurun_out/r06_t
mkdir -p $O
timeout -k 10 400 python3 -u scripts/bench_server.py --seconds 4 --batchers 2,3 > $O/serve_base.log 2>&1 || { tail -c 3000 $O/serve_base.log; exit 1; }
grep "^{" $O/serve_base.log | cut -c 1-400
timeout -k 10 400 env PILOSA_HTTP_THREAD_STREAMS=1 python3 -u scripts/bench_server.py --seconds 4 --batchers 2,3,4 > $O/serve_ts.log 2>&1 || { tail -c 3000 $O/serve_ts.log; exit 1; }
grep "^{" $O/serve_ts.log | cut -c 1-400
echo done
