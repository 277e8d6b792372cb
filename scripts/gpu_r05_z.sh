#!/bin/bash
# Round 5, call Z: 64-bit pair atomics for lane-owned hot rows, coalesced
# Min/Max fold; exactness, kernel isolation, config-4 trace.
set -o pipefail
O=gpurun_out/r05_z
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py -x -v --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_executor.py tests/test_gpu_topn_exec.py -x -q --timeout 300 --timeout-method thread -k "bsi or Sum or sum or fold or topn or TopN or slot_index" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "base:" "loadsonly:PILOSA_TOPN_DBG=4096" "noatomics:PILOSA_TOPN_DBG=256" "lanetable:PILOSA_TOPN_DBG=2064"; do
  name=${cfg%%:*}; ev=${cfg#*:}
  timeout -k 10 300 env $ev python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_$name.log 2>&1 || { tail -c 2000 $O/kb_$name.log; exit 1; }
  echo "$name: $(python3 -c "import json;d=json.loads(open('$O/kb_$name.log').read().strip().splitlines()[-1]);print({k: c['hot_ms'] for k, c in d['classes'].items()}, d.get('mix',{}).get('e2e_ms_per_batch'), d.get('mix',{}).get('parts_ms'))")"
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
python3 - <<'PY'
import sqlite3, glob
c = sqlite3.connect(glob.glob("gpurun_out/r05_z/prof_c4/*.db")[0])
for r in c.execute("select * from top_kernels limit 10"):
    print(r[0][:70], r[1], round(r[3], 1))
PY
echo done
