#!/bin/bash
# Round 5, call AO: src TopN spread with 3 untimed src requests (bench without serving / configs).
set -o pipefail
O=gpurun_out/r05_ao
mkdir -p $O
for cfg in "a:40" "b:40"; do
  name=${cfg%%:*}; nb=${cfg#*:}
  timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 5 --warmup 2 --serve-seconds 0 --configs "" --topn-batches $nb > $O/bench_$name.log 2> $O/bench_$name.err || { tail -c 3000 $O/bench_$name.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_$name.log').read().strip().splitlines()[-1]);t=d['extra']['topn'];print('$name batches $nb src', t['src'].get('qps'), t['src'].get('ms_per_request'), 'cache', t['cache'].get('qps'))"
done
echo done
