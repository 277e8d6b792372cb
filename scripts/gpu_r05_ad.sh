#!/bin/bash
# Round 5, call AD: phase-1 acc atomics isolation, then the whole GPU suite.
set -o pipefail
O=gpurun_out/r05_ad
mkdir -p $O
for cfg in "base:" "noacc:PILOSA_TOPN_DBG=8192"; do
  name=${cfg%%:*}; ev=${cfg#*:}
  timeout -k 10 300 env $ev python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_$name.log 2>&1 || { tail -c 2000 $O/kb_$name.log; exit 1; }
  echo "$name: $(python3 -c "import json;d=json.loads(open('$O/kb_$name.log').read().strip().splitlines()[-1]);print({k: (c['hot_ms'], c['phase1_ms']) for k, c in d['classes'].items()}, d.get('mix',{}).get('e2e_ms_per_batch'), d.get('mix',{}).get('parts_ms'))")"
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || { tail -c 6000 $O/pytest_all.log; exit 1; }
tail -2 $O/pytest_all.log
echo done
