#!/bin/bash
# Round 6, call R: cProfile of the world-size-1 RCCL mesh cache-only TopN
# request thread (native issue / finish), to find the host cost left.
set -o pipefail
O=gpurun_out/r06_r
mkdir -p $O
timeout -k 10 500 env PILOSA_BENCH_TOPN_PROFILE=$O/mesh_topn.folded PILOSA_BENCH_CPROFILE=$O/mesh_topn_cprofile.txt python3 -u bench.py --mesh --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
head -60 $O/mesh_topn_cprofile.txt
echo done
