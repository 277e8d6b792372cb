#!/bin/bash
# Src TopN launch width: 16-query vs 32-query hot-rank launches (NQ template),
# disk-mode index, counts/configs/serving skipped.
set -o pipefail
O=gpurun_out/r04_e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_executor.py -m gpu -q -x --timeout 200 --timeout-method thread -k "tanimoto or attr_filters" > $O/pytest_filters.log 2>&1 || { tail -c 3000 $O/pytest_filters.log; exit 1; }
tail -1 $O/pytest_filters.log
D=/tmp/pilosa_r04e
for cfg in "16 16" "16 32" "32 32"; do
  set -- $cfg
  timeout -k 10 600 env PILOSA_TOPN_HOT_Q=$2 python -u bench.py --steps 2 --warmup 1 --configs none --serve-seconds 0 \
      --topn-batch $1 --topn-batches 40 --data-dir $D --keep-data > $O/bench_b$1_q$2.log 2> $O/bench_b$1_q$2.err \
      || { tail -c 2000 $O/bench_b$1_q$2.err; exit 1; }
  python - "$O/bench_b$1_q$2.log" "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"]["topn"]
print("batch", sys.argv[2], "hot_q", sys.argv[3], "src", t["src"].get("qps"), t["src"].get("ms_per_request"),
      "cache", t["cache"].get("qps"), "verified", t.get("verify", {}).get("verified"))
PY
done
