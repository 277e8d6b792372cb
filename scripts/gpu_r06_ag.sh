#!/bin/bash
# Round 6, call AG: src TopN fixed costs -- no has-run flag read when the arena has no run containers
# (after call AF: host finish, searchsorted offsets):
# TopN GPU tests, kernel-level batch at 954 and 120 shards, bench src phase.
set -o pipefail
O=gpurun_out/r06_ag
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_topn_exec.py tests/test_gpu_mesh.py tests/test_gpu_rccl_mesh.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 1000000000 125000000; do
  timeout -k 10 300 env PILOSA_HIPKERNELS=_hipkernels python3 -u scripts/topn_kbench.py --reps 10 --cols $c > $O/kb_$c.log 2>&1 || { tail -20 $O/kb_$c.log; exit 1; }
  grep "^{" $O/kb_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cols $c shards', d['shards'], d['mix'])"
done
timeout -k 10 500 python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_ag/bench.log") if l.startswith("{")][-1])
t = d["extra"]["topn"]
print(d["value"], {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v}, t.get("src", {}).get("single_thread_ms_per_request"), t.get("verify"))
PY
echo done
