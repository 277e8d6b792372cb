#!/bin/bash
# Round 6, call N: src TopN operating point after the carry-save rewrite:
# hot-rank count (PILOSA_TOPN_HOT) x lane-owned bound (PILOSA_TOPN_SMALL_N),
# batch time of the bench mix (topn_kbench, shipped kernels).
set -o pipefail
O=gpurun_out/r06_n
mkdir -p $O
for cfg in "3072 255" "2048 255" "2560 255" "3584 255" "4096 255" "3072 63" "3072 1023" "2560 1023"; do
  set -- $cfg
  timeout -k 10 300 env PILOSA_HIPKERNELS=_hipkernels PILOSA_TOPN_HOT=$1 PILOSA_TOPN_SMALL_N=$2 python3 -u scripts/topn_kbench.py --reps 5 > $O/kb_$1_$2.log 2>&1 || { tail -20 $O/kb_$1_$2.log; exit 1; }
  grep "^{" $O/kb_$1_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); m=d['mix']; print('hot $1 small $2', m['e2e_ms_per_batch'], m['qps'], m['parts_ms'])"
done
echo done
