#!/bin/bash
# hot-rank kernel cost isolation: PILOSA_TOPN_DBG 8 = no small path, 16 = no big path, 24 = table only
set -o pipefail
mkdir -p gpurun_out
for d in 0 8 16 24; do
  for src in 0 900; do
    PILOSA_TOPN_DBG=$d timeout -k 10 200 python -u scripts/topn_hot_probe.py --shards 256 --src $src > gpurun_out/tprobe.log 2>&1 || { tail -20 gpurun_out/tprobe.log; exit 1; }
    echo "dbg=$d src=$src $(tail -1 gpurun_out/tprobe.log)"
  done
done
