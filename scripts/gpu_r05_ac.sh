#!/bin/bash
# Round 5, call AC: array-src table build over the whole workgroup; exactness,
# kernel timing, then the driver's bench.
set -o pipefail
O=gpurun_out/r05_ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py tests/test_gpu_topn_exec.py -x -q --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
timeout -k 10 300 python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_base.log 2>&1 || { tail -c 2000 $O/kb_base.log; exit 1; }
timeout -k 10 300 env PILOSA_TOPN_DBG=8192 python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_noacc.log 2>&1 || { tail -c 2000 $O/kb_noacc.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/kb_noacc.log').read().strip().splitlines()[-1]);print('noacc phase1', {k: c['phase1_ms'] for k, c in d['classes'].items()})"
timeout -k 10 300 env PILOSA_TOPN_DBG=2072 python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_tableonly.log 2>&1 || { tail -c 2000 $O/kb_tableonly.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/kb_tableonly.log').read().strip().splitlines()[-1]);print('tableonly', {k: c['hot_ms'] for k, c in d['classes'].items()})"
python3 -c "import json;d=json.loads(open('$O/kb_base.log').read().strip().splitlines()[-1]);print({k: (c['hot_ms'], c['phase1_ms']) for k, c in d['classes'].items()}, d.get('mix',{}))"
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05_ac/bench.log").read().strip().splitlines()[-1])
ex = d["extra"]
print("headline", d["value"])
print("topn", {k: v.get("qps") for k, v in ex["topn"].items() if isinstance(v, dict)})
print("serving", ex["serving"]["count"]["req_per_s"], ex["serving"]["count"]["p99_ms"], ex["serving"]["count_topn_mix"]["req_per_s"], ex["serving"]["count_topn_mix"]["p99_ms"])
print("bsi", {k: v["ms_per_request"] for k, v in ex["config4_bsi"]["queries"].items()})
print("config5", ex["config5_time_union"]["qps"])
PY
echo done
