#!/bin/bash
# Round 6, call AJ: serving Count with 32 queries per wave for 33-64-query
# batches: pair-kernel GPU tests, then the serving bench twice.
set -o pipefail
O=gpurun_out/r06_aj
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_executor.py > $O/pytest.log 2>&1 || { tail -c 4000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/bench_server.py --seconds 4 --batchers 2 > $O/serve_$r.log 2>&1 || { tail -c 3000 $O/serve_$r.log; exit 1; }
  grep "^{" $O/serve_$r.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d.get('server_stats',{})
    print('run $r', d['value'], 'p99', d['p99_ms'], 'req/batch', round(s.get('batched_requests',0)/max(1,s.get('batches',1)),1), 'mismatch', d.get('mismatches'))"
done
echo done
