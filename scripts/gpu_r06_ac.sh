#!/bin/bash
# Round 6, call AC: adaptive group commit for serving Count -- while another
# batch is on the device a batcher waits up to HOLD_US for HOLD_MIN requests.
set -o pipefail
O=gpurun_out/r06_ac
mkdir -p $O
for cfg in "0 0 2" "64 300 2" "96 400 2" "112 600 2" "80 200 2" "64 300 3"; do
  set -- $cfg
  timeout -k 10 300 env PILOSA_HTTP_HOLD_MIN=$1 PILOSA_HTTP_HOLD_US=$2 python3 -u scripts/bench_server.py --seconds 4 --batchers $3 > $O/serve_$1_$2_$3.log 2>&1 || { tail -c 3000 $O/serve_$1_$2_$3.log; exit 1; }
  grep "^{" $O/serve_$1_$2_$3.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); s=d.get('server_stats',{})
    print('hold $1 $2 batchers $3', d['value'], 'p99', d['p99_ms'], 'req/batch', round(s.get('batched_requests',0)/max(1,s.get('batches',1)),1), 'held', s.get('held_batches'), 'mismatch', d.get('mismatches'))"
done
echo done
