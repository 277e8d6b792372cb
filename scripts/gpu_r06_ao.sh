#!/bin/bash
# Round 6, call AO: PMC of the src TopN kernels after the flat phase-1
# histogram (phase 1 and the hot-rank kernel), one counter set per pass.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_ao
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $SET --kernel-include-regex "topn_hot_kernel|topn_src_kernel" --output-format csv -d $O/pmc -o set$i -- python3 $R/scripts/topn_kbench.py --reps 1 > $O/pmc_set$i.log 2>&1 || { tail -20 $O/pmc_set$i.log; exit 1; }
  echo "pass $i done"
done
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/r06_ao/pmc/set*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    g = lambda n: d.get(n, 0.0)
    print(k)
    if g("SQ_LDS_IDX_ACTIVE"): print("  lds_conflict/active", round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 3))
    if g("SQ_WAVE_CYCLES"): print("  wait_any/wave_cycles", round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 3), "valu/wave_cycles", round(g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES"), 3))
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"): print("  l2_hit", round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 3))
PY
echo done
