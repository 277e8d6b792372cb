#!/bin/bash
# Round 5, call AE: src TopN request threads (bench.py without serving / configs).
set -o pipefail
O=gpurun_out/r05_ae
mkdir -p $O
for c in 2 3 4 6; do
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --serve-seconds 0 --configs "" --topn-clients $c > $O/bench_c$c.log 2> $O/bench_c$c.err || { tail -c 3000 $O/bench_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_c$c.log').read().strip().splitlines()[-1]);t=d['extra']['topn'];print('clients $c', t['src'].get('qps'), t['src'].get('ms_per_request'), t['cache'].get('qps'))"
done
echo done
