#!/bin/bash
# Round 6, call AP: phase-1 fill walk with one barrier per chunk (ranked pass only where the heap fills)
# (after the flat histogram of call V): src TopN GPU tests, kernel-level batch
# (shipped module), then the bench's src phase.
set -o pipefail
O=gpurun_out/r06_ap
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_topn_exec.py tests/test_gpu_hot_counts.py tests/test_gpu_executor.py tests/test_gpu_shardwidth.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 env PILOSA_HIPKERNELS=_hipkernels python3 -u scripts/topn_kbench.py --reps 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep "^{" $O/kb.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: (v['hot_ms'], v['phase1_ms']) for k, v in d['classes'].items()}, d['mix'])"
timeout -k 10 500 python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_ap/bench.log") if l.startswith("{")][-1])
t = d["extra"]["topn"]
print(d["value"], {k: (v.get("qps"), v.get("ms_per_request"), v.get("p50_ms"), v.get("p99_ms")) for k, v in t.items() if isinstance(v, dict) and "qps" in v}, t.get("src", {}).get("single_thread_ms_per_request"))
PY
echo done
