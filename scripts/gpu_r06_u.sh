#!/bin/bash
# Round 6, call U: phase-1 (topn_src_kernel<1>) attribution per src class:
# PILOSA_TOPN_DBG=2 skips the heap walk, =1 the tail histogram (kbench module).
set -o pipefail
O=gpurun_out/r06_u
mkdir -p $O
for d in 0 2 1; do
  timeout -k 10 300 env PILOSA_TOPN_DBG=$d python3 -u scripts/topn_kbench.py --reps 5 > $O/kb_dbg$d.log 2>&1 || { tail -20 $O/kb_dbg$d.log; exit 1; }
  grep "^{" $O/kb_dbg$d.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dbg $d', {k: (v['hot_ms'], v['phase1_ms']) for k, v in d['classes'].items()}, d.get('mix', {}).get('parts_ms'))"
done
echo done
