#!/bin/bash
# Round 6, call AQ: cProfile of the world-size-1 RCCL mesh src TopN request
# thread (one thread), to find the ~1 ms per request above the plain path.
set -o pipefail
O=gpurun_out/r06_aq
mkdir -p $O
timeout -k 10 600 env PILOSA_BENCH_TOPN_SRC_PROFILE=$O/mesh_src.folded PILOSA_BENCH_CPROFILE=$O/mesh_src_cprofile.txt python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 60 --topn-clients 1 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
head -70 $O/mesh_src_cprofile.txt
echo done
