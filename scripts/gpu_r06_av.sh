#!/bin/bash
# Round 6, call AV: cache-only batch with membership + totals in one launch and an
# epoch-marked member buffer (no clear per batch): tests, bench, kernel stats.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_av
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_topn_exec.py tests/test_gpu_rccl_mesh.py tests/test_gpu_mesh.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r06_av/bench.log") if l.startswith("{")][-1])
t = d["extra"]["topn"]
print(d["value"], {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v}, t.get("verify"))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o av -- python3 $R/bench.py --serve-seconds 0 --configs= --steps 2 --warmup 1 --topn-src-batches 8 > $O/bench_prof.log 2> $O/bench_prof.err || { tail -c 3000 $O/bench_prof.err; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
grep -i "topn_cache" $f | cut -c 1-260
echo done
