#!/bin/bash
# Round 5, call V: transposed-build threshold sweep on the bench mix, and
# per-path PMC counters of the hot-rank kernel (PILOSA_TOPN_DBG isolation).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r05_v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot_counts.py -x -q --timeout 300 --timeout-method thread -k "not every_bound" > $O/pytest_hot.log 2>&1 || { tail -c 5000 $O/pytest_hot.log; exit 1; }
tail -1 $O/pytest_hot.log
for tb in 4097 12288 24576 70000; do
  timeout -k 10 300 env PILOSA_TOPN_TBUILD_MIN=$tb python3 -u scripts/topn_kbench.py --reps 3 > $O/kb_tb$tb.log 2>&1 || { tail -c 2000 $O/kb_tb$tb.log; exit 1; }
  echo "tb$tb: $(python3 -c "import json;d=json.loads(open('$O/kb_tb$tb.log').read().strip().splitlines()[-1]);print([c['hot_ms'] for c in d['classes'].values()], d['mix']['e2e_ms_per_batch'], d['mix']['parts_ms']['hot'])")"
done
cd /tmp && export TMPDIR=/tmp
for dbg in 0 8 16; do
  i=0
  for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
    i=$((i+1))
    PILOSA_TOPN_DBG=$dbg timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "topn_hot_kernel" --output-format csv -d $O/pmc_d$dbg -o set$i -- python3 $R/scripts/topn_hot_probe.py --shards 128 --reps 1 --src mix > $O/pmc_d${dbg}_set$i.log 2>&1 || { tail -20 $O/pmc_d${dbg}_set$i.log; exit 1; }
  done
done
cd $R && python3 - <<'PY' > gpurun_out/r05_v/pmc_summary.txt
import csv, glob, collections
for d in ("0", "8", "16"):
    agg = collections.defaultdict(float)
    for f in sorted(glob.glob(f"gpurun_out/r05_v/pmc_d{d}/**/set*_counter_collection.csv", recursive=True)):
        rows = list(csv.DictReader(open(f)))
        disp = sorted(set(r["Dispatch_Id"] for r in rows))[-1:]   # the timed launch
        for r in rows:
            if r["Dispatch_Id"] in disp:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print("dbg", d)
    for c, v in sorted(agg.items()):
        print(f"  {c:28s} {v:.4g}")
PY
cat gpurun_out/r05_v/pmc_summary.txt
echo done
