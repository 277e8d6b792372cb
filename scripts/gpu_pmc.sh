#!/bin/bash
# PMC counter passes over the kernel harness (one rocprofv3 run per counter set).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmc
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
KRE=${KRE:-and2_pairs}
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$KRE" --output-format csv -d $R/gpurun_out/pmc -o set$i -- python3 $R/scripts/kbench.py --reps 1 --cq ${CQ:-8} ${KB_ARGS} > $R/gpurun_out/pmc/set$i.log 2>&1 || { tail -20 $R/gpurun_out/pmc/set$i.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/pmc/set*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:.4g}")
PY
