#!/bin/bash
# Round 5, call E: TopN correctness after the columnar-result / batch-memo
# changes, the cache-only request profile again (local vs world-1 mesh), and
# a kernel trace of config 4 (BSI Sum / range / Min / Max).
set -o pipefail
R=$PWD
O=gpurun_out/r05_e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_mesh.py tests/test_gpu_rccl_mesh.py tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 6000 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python -u scripts/prof_topn_paths.py --reqs 300 > $O/prof_topn.log 2>&1 || { tail -c 3000 $O/prof_topn.log; exit 1; }
grep -E "requests x|mesh data" $O/prof_topn.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/c4 -o c4 -- python3 $R/scripts/prof_configs.py --which 4 --reps 20 > $R/$O/prof_c4.log 2>&1 || { tail -c 3000 $R/$O/prof_c4.log; exit 1; }
cd $R
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05_e/c4/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms tot")
PY
grep -o '"queries": {.*}, "device' $O/prof_c4.log | head -c 1500
