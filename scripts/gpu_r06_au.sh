#!/bin/bash
# Round 6, call AU: cProfile of the plain cache-only TopN request thread
# after the native request object (what Python is left per request).
set -o pipefail
O=gpurun_out/r06_au
mkdir -p $O
timeout -k 10 500 env PILOSA_BENCH_TOPN_PROFILE=$O/plain_topn.folded PILOSA_BENCH_CPROFILE=$O/plain_topn_cprofile.txt python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
head -50 $O/plain_topn_cprofile.txt
echo done
