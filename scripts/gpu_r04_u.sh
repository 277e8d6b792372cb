#!/bin/bash
# BSI kernels: GPU executor suite, then config 4 with min/max at 2 and 3 waves per SIMD.
set -o pipefail
O=gpurun_out/r04_u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_executor.py -m gpu -q -x --timeout 500 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 3000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
D=/tmp/pilosa_r04u
for W in 2 3; do
  timeout -k 10 700 env PILOSA_BSI_MINMAX_WAVES=$W python -u bench.py --steps 2 --warmup 1 --configs 4 --serve-seconds 0 --topn-batches 0 \
      --data-dir $D --keep-data > $O/bench_w$W.log 2> $O/bench_w$W.err || { tail -c 2000 $O/bench_w$W.err; exit 1; }
  python - "$O/bench_w$W.log" "$W" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
q = d["extra"].get("config4_bsi", {}).get("queries", {})
print("waves", sys.argv[2], {k: (v.get("ms_per_request"), v.get("sample")) for k, v in q.items()})
PY
done
