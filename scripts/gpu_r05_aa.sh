#!/bin/bash
# Round 5, call AA: the whole GPU suite after the hot-kernel / BSI changes,
# then the bench-mix kernel timing.
set -o pipefail
O=gpurun_out/r05_aa
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || { tail -c 6000 $O/pytest_all.log; exit 1; }
tail -2 $O/pytest_all.log
timeout -k 10 300 python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_base.log 2>&1 || { tail -c 2000 $O/kb_base.log; exit 1; }
python3 -c "import json;d=json.loads(open('$O/kb_base.log').read().strip().splitlines()[-1]);print({k: c['hot_ms'] for k, c in d['classes'].items()}, d.get('mix',{}))"
echo done
