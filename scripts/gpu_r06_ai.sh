#!/bin/bash
# Round 6, call AI: serving-size pair kernel at wider chunks (32 / 64 queries
# per wave: one wave per unit holds every same-A run of a sorted batch); then
# the plain TopN fast path keyed on the shard epoch (tests + bench phases).
set -o pipefail
O=gpurun_out/r06_ai
mkdir -p $O
for B in 64 128; do
  timeout -k 10 300 python3 -u scripts/kbench.py --batch $B --reps 30 --cq "" --no-tile \
    --variants 39@16,39@32,39@64,6@32,6@64 > $O/kbench_b$B.log 2>&1 || { tail -30 $O/kbench_b$B.log; exit 1; }
  echo "batch $B"; grep -v "^{" $O/kbench_b$B.log | grep and2
done
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_topn_exec.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_ai/bench.log") if l.startswith("{")][-1])
t = d["extra"]["topn"]
print(d["value"], {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v}, t.get("verify"))
PY
echo done
