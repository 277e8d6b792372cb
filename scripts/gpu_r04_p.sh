#!/bin/bash
# Src TopN: hot-rank count R (PILOSA_TOPN_HOT) sweep through the bench's TopN phase.
set -o pipefail
O=gpurun_out/r04_p
mkdir -p $O
D=/tmp/pilosa_r04p
for R in ${RS:-2048 2560 3072 3584}; do
  timeout -k 10 600 env PILOSA_TOPN_HOT=$R python -u bench.py --steps 2 --warmup 1 --configs none --serve-seconds 0 \
      --topn-batches 40 --topn-cache-batches 40 --data-dir $D --keep-data > $O/bench_R$R.log 2> $O/bench_R$R.err \
      || { tail -c 2000 $O/bench_R$R.err; exit 1; }
  python - "$O/bench_R$R.log" "$R" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"]["topn"]
print("R", sys.argv[2], "src", t["src"].get("qps"), t["src"].get("ms_per_request"), "verified", t.get("verify", {}).get("verified"))
PY
done
