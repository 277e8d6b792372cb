#!/bin/bash
# Serving phase only (count, count+TopN mix, import) with the server's stacks
# sampled during the mix.
set -o pipefail
O=gpurun_out/r04_g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topn_exec.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_topn.log 2>&1 || { tail -c 3000 $O/pytest_topn.log; exit 1; }
tail -1 $O/pytest_topn.log
timeout -k 10 900 python -u bench.py --steps 2 --warmup 1 --topn-batches 0 --configs none --serve-seconds 6 \
    --serve-profile $O/mix_profile.txt > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04_g/bench.log") if l.startswith("{")][-1])
s = d["extra"]["serving"]
print(json.dumps({k: s[k] for k in ("count", "count_topn_mix", "import")})[:1500])
PY
