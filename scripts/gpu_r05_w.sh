#!/bin/bash
# Round 5, call W: quarter-wave path for mid-size hot rows; BSI Sum split of
# consider by sign.  Exactness (dense reference at every bound, executor
# suites), kernel timing, bench-mix TopN, config 4 under a kernel trace.
set -o pipefail
O=gpurun_out/r05_w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py -x -v --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread -k "slot_index or topn or TopN or bsi or Sum" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "base:" "nomid:PILOSA_TOPN_MID_N=0" "mid512:PILOSA_TOPN_MID_N=512" "nomidrows:PILOSA_TOPN_DBG=2048"; do
  name=${cfg%%:*}; ev=${cfg#*:}
  timeout -k 10 300 env $ev python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_$name.log 2>&1 || { tail -c 2000 $O/kb_$name.log; exit 1; }
  echo "$name: $(python3 -c "import json;d=json.loads(open('$O/kb_$name.log').read().strip().splitlines()[-1]);print([c['hot_ms'] for c in d['classes'].values()], d.get('mix',{}).get('e2e_ms_per_batch'), d.get('mix',{}).get('parts_ms',{}).get('hot'))")"
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
grep -E "sum|range|min|max" $O/prof_c4.log | tail -8
echo done
