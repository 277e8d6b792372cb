#!/bin/bash
# Hot-rank TopN kernel: lane-owned containers up to 255 (default) vs 1023 values;
# cache-only TopN batches on per-thread side streams vs the current stream.
set -o pipefail
O=gpurun_out/r04_h
mkdir -p $O
timeout -k 10 620 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py tests/test_gpu_shardwidth.py -m gpu -q -x --timeout 600 --timeout-method thread -k "not narrow_width and not wide_width" > $O/pytest_small.log 2>&1 || { tail -c 3000 $O/pytest_small.log; exit 1; }
tail -1 $O/pytest_small.log
D=/tmp/pilosa_r04h
for v in 255:1 1023:1 255:0; do
  sn=${v%:*}; ss=${v#*:}
  timeout -k 10 600 env PILOSA_TOPN_SMALL_N=$sn PILOSA_TOPN_SIDE_STREAM=$ss python -u bench.py --steps 2 --warmup 1 --configs none --serve-seconds 0 \
      --topn-batches 40 --data-dir $D --keep-data > $O/bench_sn${sn}_ss$ss.log 2> $O/bench_sn${sn}_ss$ss.err \
      || { tail -c 2000 $O/bench_sn${sn}_ss$ss.err; exit 1; }
  python - "$O/bench_sn${sn}_ss$ss.log" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"]["topn"]
print("small_n:side", sys.argv[2], "src", t["src"].get("qps"), t["src"].get("ms_per_request"),
      "cache", t["cache"].get("qps"), "verified", t.get("verify", {}).get("verified"))
PY
done
