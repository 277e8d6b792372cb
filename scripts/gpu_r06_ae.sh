#!/bin/bash
# Round 6, call AE: the src TopN batch on one rank's share of an N-GPU node
# (954 / N shards: --cols 1e9 / N), kernel-level, to see the fixed per-batch
# costs the 8-GPU curve will pay.
set -o pipefail
O=gpurun_out/r06_ae
mkdir -p $O
for c in 1000000000 500000000 250000000 125000000; do
  timeout -k 10 300 env PILOSA_HIPKERNELS=_hipkernels python3 -u scripts/topn_kbench.py --reps 10 --cols $c > $O/kb_$c.log 2>&1 || { tail -20 $O/kb_$c.log; exit 1; }
  grep "^{" $O/kb_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cols $c shards', d['shards'], d['mix'])"
done
echo done
