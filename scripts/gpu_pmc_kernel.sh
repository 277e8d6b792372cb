#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter set) over one kernel of a
# harness: KRE = kernel regex, CMD = harness command (python script + args).
set -o pipefail
R=$PWD
OUT=${OUT:-gpurun_out/pmc_k}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "$KRE" --output-format csv -d $R/$OUT -o set$i -- python3 $R/$CMD > $R/$OUT/set$i.log 2>&1 || { tail -20 $R/$OUT/set$i.log; exit 1; }
  echo "pass $i done"
done
cd $R && OUT=$OUT python3 - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(os.environ["OUT"] + "/**/set*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:.4g}")
    g = lambda n: d.get(n, 0.0)
    if g("SQ_WAVE_CYCLES"):
        print(f"  wait_any/wave_cycles      {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
        print(f"  active_inst/wave_cycles   {g('SQ_ACTIVE_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_INSTS_VALU"):
        print(f"  salu/valu                 {g('SQ_INSTS_SALU') / g('SQ_INSTS_VALU'):.3f}")
    if g("SQ_LDS_IDX_ACTIVE"):
        print(f"  lds_bank_conflict/active  {g('SQ_LDS_BANK_CONFLICT') / g('SQ_LDS_IDX_ACTIVE'):.3f}")
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"):
        print(f"  l2_hit                    {g('TCC_HIT_sum') / (g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
PY
