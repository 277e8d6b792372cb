#!/bin/bash
# PMC counter passes over the pair kernel variants (v6/v7/v8), 4096-query
# Count(Intersect) batch on the config-2 arena, one rocprofv3 run per counter set.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/pmc3
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "and2_pairs_v[678]" --output-format csv -d $R/gpurun_out/pmc3 -o set$i -- python3 $R/scripts/kbench.py --reps 1 --cq "" --variants ${VARIANTS:-6,7,8} --no-tile --batch 4096 > $R/gpurun_out/pmc3/set$i.log 2>&1 || { tail -20 $R/gpurun_out/pmc3/set$i.log; exit 1; }
  echo "pass $i done"
done
cd $R && python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/pmc3/set*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:.4g}")
    g = lambda n: d.get(n, 0.0)
    if g("SQ_WAVE_CYCLES"):
        print(f"  wait_any/wave_cycles      {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_INSTS_VALU"):
        print(f"  salu/valu                 {g('SQ_INSTS_SALU') / g('SQ_INSTS_VALU'):.3f}")
    if g("SQ_LDS_IDX_ACTIVE"):
        print(f"  lds_bank_conflict/active  {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        print(f"  l2_hit                    {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
PY
