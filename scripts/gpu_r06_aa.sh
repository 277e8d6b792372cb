#!/bin/bash
# Round 6, call AA: kernel trace of the bench's headline + TopN phases from
# the FIRST bench process on a fresh box, per-kernel stats.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o first -- python3 $R/bench.py --serve-seconds 0 --configs= --steps 5 --warmup 2 > $O/bench_first.log 2> $O/bench_first.err || { tail -c 3000 $O/bench_first.err; exit 1; }
cd $R
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
echo $f
head -25 $f | cut -c 1-200
python3 - $O/bench_first.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["extra"]["topn"]
print(d["value"], {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v})
PY
echo done
# kernel-level src batch at 16 / 32 queries (the hot-rank kernel's NQ = 32
# half-key mode streams the same bytes for twice the queries)
for b in 16 32; do
  timeout -k 10 300 env PILOSA_HIPKERNELS=_hipkernels python3 -u scripts/topn_kbench.py --reps 5 --batch $b > $O/kb_b$b.log 2>&1 || { tail -20 $O/kb_b$b.log; exit 1; }
  grep "^{" $O/kb_b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('batch $b', {k: (v['hot_ms'], v['phase1_ms']) for k, v in d['classes'].items()}, d['mix'])"
done
echo done2
