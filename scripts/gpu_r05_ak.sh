#!/bin/bash
# Round 5, call AK: multi-block Min/Max fold (exactness, config-4 trace),
# then the 4-rank gloo rehearsal on the final code.
set -o pipefail
O=gpurun_out/r05_ak
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread -k "fold or bsi or Min or Max" > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
python3 - <<'PY'
import sqlite3, glob
c = sqlite3.connect(glob.glob("gpurun_out/r05_ak/prof_c4/*.db")[0])
for r in c.execute("select * from top_kernels limit 12"):
    print(r[0][:70], r[1], round(r[3], 1))
PY
grep -i "min\|max" $O/prof_c4.log | tail -4
bash scripts/gpu_r05_aj.sh
echo done
