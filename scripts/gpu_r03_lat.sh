#!/bin/bash
# Latency counters (Little's law: SQ_INST_LEVEL_x / SQ_INSTS_x = mean cycles in
# flight) of the shipped pair kernel, plus the counter list of the box.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r03_lat
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/r03_lat/counters.txt 2>&1 || true
(cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_gpu_topn_exec.py > $R/gpurun_out/r03_lat/pytest_topn.log 2>&1) || { tail -c 2000 $R/gpurun_out/r03_lat/pytest_topn.log; exit 1; }
tail -2 $R/gpurun_out/r03_lat/pytest_topn.log
i=0
for SET in "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM" \
           "TA_BUSY_avr TA_TA_BUSY_sum TD_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "and2_pairs_v6" --output-format csv -d $R/gpurun_out/r03_lat -o set$i -- python3 $R/scripts/kbench.py --reps 1 --cq 64 --no-tile --batch 4096 > $R/gpurun_out/r03_lat/set$i.log 2>&1 || { tail -5 $R/gpurun_out/r03_lat/set$i.log; echo "pass $i failed"; continue; }
  echo "pass $i done"
done
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/r03_lat/**/set*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:.4g}")
PY
grep -i "LEVEL\|TA_BUSY\|TD_BUSY\|TCP_PENDING\|TCC_EA0_RDREQ_LEVEL\|TCC_EA0_RD_UNCACHED\|MALL\|TCC_EA0_RDREQ_DRAM" gpurun_out/r03_lat/counters.txt | head -60
