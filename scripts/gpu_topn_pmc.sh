#!/bin/bash
# PMC passes over the hot-rank TopN kernel (scripts/topn_hot_probe.py).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/tpmc
timeout -k 10 200 python -u scripts/topn_hot_probe.py --shards 128 --src ${SRC:-900} > gpurun_out/tpmc/probe.log 2>&1 || { tail -20 gpurun_out/tpmc/probe.log; exit 1; }
tail -1 gpurun_out/tpmc/probe.log
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $SET --kernel-include-regex "topn_hot_kernel" --output-format csv -d $R/gpurun_out/tpmc -o set$i -- python3 $R/scripts/topn_hot_probe.py --shards 128 --reps 1 --src ${SRC:-900} > $R/gpurun_out/tpmc/set$i.log 2>&1 || { tail -20 $R/gpurun_out/tpmc/set$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/tpmc/**/set*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:.4g}")
PY
