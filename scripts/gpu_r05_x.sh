#!/bin/bash
# Round 5, call X: mid-size bound sweep (1024 / 2048) for the hot-rank TopN
# kernel; BSI Sum with one atomic pair per block; then the driver's bench.
set -o pipefail
O=gpurun_out/r05_x
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_hot_counts.py -x -v --timeout 600 --timeout-method thread > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_executor.py -x -q --timeout 300 --timeout-method thread -k "bsi or Sum or sum" > $O/pytest_bsi.log 2>&1 || { tail -c 5000 $O/pytest_bsi.log; exit 1; }
tail -1 $O/pytest_bsi.log
for cfg in "base:" "mid2048:PILOSA_TOPN_MID_N=2048" "small63:PILOSA_TOPN_SMALL_N=63" "hot4096:PILOSA_TOPN_HOT=4096" "hot2048:PILOSA_TOPN_HOT=2048"; do
  name=${cfg%%:*}; ev=${cfg#*:}
  timeout -k 10 300 env $ev python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_$name.log 2>&1 || { tail -c 2000 $O/kb_$name.log; exit 1; }
  echo "$name: $(python3 -c "import json;d=json.loads(open('$O/kb_$name.log').read().strip().splitlines()[-1]);print([c['hot_ms'] for c in d['classes'].values()], d.get('mix',{}).get('e2e_ms_per_batch'), d.get('mix',{}).get('parts_ms',{}).get('hot'))")"
done
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 -u scripts/prof_configs.py --which 4 --reps 20 --no-profile > $O/prof_c4.log 2>&1 || { tail -c 3000 $O/prof_c4.log; exit 1; }
timeout -k 10 900 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
tail -c 1500 $O/bench.log
echo done
