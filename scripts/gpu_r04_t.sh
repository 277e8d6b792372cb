#!/bin/bash
# BSI Min/Max: which-specific descents. GPU executor suite, then config 4 through the bench.
set -o pipefail
O=gpurun_out/${OUT:-r04_t}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_executor.py -m gpu -q -x --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 3000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 700 python -u bench.py --steps 2 --warmup 1 --configs 4 --serve-seconds 0 --topn-batches 0 > $O/bench.log 2> $O/bench.err || { tail -c 2000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/" + __import__("os").environ.get("OUT", "r04_t") + "/bench.log") if l.startswith("{")][-1])
print(json.dumps(d["extra"].get("config4_bsi", {}).get("queries"))[:900])
PY
