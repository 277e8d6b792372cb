#!/bin/bash
# Hot-rank TopN kernel cost isolation (PILOSA_TOPN_DBG): 0 = full,
# 24 = mask-table build only, 8 = no small rows, 16 = no big rows,
# 32 = big rows without bitmap containers, 64 = big rows without arrays.
set -o pipefail
mkdir -p gpurun_out/r03_hotiso
for d in 0 24 8 16 32 64; do
  PILOSA_TOPN_DBG=$d timeout -k 10 300 python -u scripts/topn_kbench.py --reps 5 > gpurun_out/r03_hotiso/dbg$d.log 2>&1 || { tail -c 2000 gpurun_out/r03_hotiso/dbg$d.log; exit 1; }
  echo "dbg=$d $(grep '^{' gpurun_out/r03_hotiso/dbg$d.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: v["hot_ms"] for k, v in d["classes"].items()}, d.get("mix", {}).get("parts_ms"))')"
done
