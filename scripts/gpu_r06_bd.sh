#!/bin/bash
# Round 6, call BD: rank-cache re-ranks bump the mutation epoch (device memo served a pre-re-rank
# ranking: the width-18 slot-index mismatch of calls AZ/BB/BC). Width-18 TopN module, the whole GPU
# suite, smoke; then bench --mesh with the all-reduce on the caller's stream vs the process group's.
set -o pipefail
O=gpurun_out/r06_bd
mkdir -p $O
PILOSA_SHARD_WIDTH=18 timeout -k 10 300 python3 -u -m pytest -x -s -q -p no:cacheprovider -m gpu --timeout 200 --timeout-method thread tests/test_gpu_topn_exec.py > $O/width18_topn.log 2>&1 || { grep -E "SLOTDIFF|SLOTROW" $O/width18_topn.log | cut -c1-1500; tail -c 3000 $O/width18_topn.log; exit 1; }
tail -1 $O/width18_topn.log
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_all.log 2>&1 || { tail -c 4000 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -c 3000 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
D=/tmp/pilosa_bd_data
for m in current pg; do
  PILOSA_MESH_AR_STREAM=$m timeout -k 10 240 python3 -u bench.py --mesh --serve-seconds 0 --configs "" --topn-pairs-batches 0 --data-dir $D --keep-data > $O/bench_mesh_$m.log 2> $O/bench_mesh_$m.err || { tail -c 2000 $O/bench_mesh_$m.err; exit 1; }
  python3 - $O/bench_mesh_$m.log $m <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"].get("topn", {})
print(sys.argv[2], "value", d["value"], "verified", d.get("verified"), "topn", {k: (t.get(k) or {}).get("qps") for k in ("cache", "cache_cycling", "cache_repeated", "src")})
PY
done
echo done
