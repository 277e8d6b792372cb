#!/bin/bash
# Round 5, call AG: quarter-wave first chunks a quad ahead;
# exactness, kernel timing, src TopN in the bench (no serving / configs).
set -o pipefail
O=gpurun_out/r05_ag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py tests/test_gpu_topn_exec.py -x -q --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
timeout -k 10 300 python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_base.log 2>&1 || { tail -c 2000 $O/kb_base.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/kb_base.log').read().strip().splitlines()[-1]);print({k: (c['hot_ms'], c['phase1_ms']) for k, c in d['classes'].items()}, d.get('mix',{}))"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --serve-seconds 0 --configs "" > $O/bench_topn.log 2> $O/bench_topn.err || { tail -c 3000 $O/bench_topn.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_topn.log').read().strip().splitlines()[-1]);t=d['extra']['topn'];print('src', t['src'].get('qps'), t['src'].get('ms_per_request'), 'cache', t['cache'].get('qps'))"
echo done
