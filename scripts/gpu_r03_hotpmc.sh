#!/bin/bash
# PMC passes over the hot-rank TopN kernel (topn_hot_kernel<16>) on the
# headline arena (scripts/topn_kbench.py --reps 1): where its time goes
# (VALU vs LDS vs memory waits), one counter set per run.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r03_hotpmc
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "topn_hot_kernel" --output-format csv -d $R/gpurun_out/r03_hotpmc -o set$i -- python3 $R/scripts/topn_kbench.py --reps 1 > $R/gpurun_out/r03_hotpmc/set$i.log 2>&1 || { tail -20 $R/gpurun_out/r03_hotpmc/set$i.log; exit 1; }
  echo "pass $i done"
done
cd $R && python3 - <<'PY'
import csv, glob, collections
d = collections.defaultdict(float)
n = collections.defaultdict(int)
for f in sorted(glob.glob("gpurun_out/r03_hotpmc/**/set*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
for c in sorted(d):
    print(f"  {c:24s} {d[c]:.4g}")
g = d.get
print("wait_any/wave_cycles", round(g("SQ_WAIT_ANY", 0) / max(1, g("SQ_WAVE_CYCLES", 1)), 3))
print("active_valu/busy_cycles(per SIMD est)", round(g("SQ_ACTIVE_INST_VALU", 0) / max(1, g("SQ_BUSY_CYCLES", 1)), 3))
print("active_lds/busy", round(g("SQ_ACTIVE_INST_LDS", 0) / max(1, g("SQ_BUSY_CYCLES", 1)), 3))
print("lds_bank_conflict/lds_idx_active", round(g("SQ_LDS_BANK_CONFLICT", 0) / max(1, g("SQ_LDS_IDX_ACTIVE", 1)), 3))
print("valu insts per lds inst", round(g("SQ_INSTS_VALU", 0) / max(1, g("SQ_INSTS_LDS", 1)), 2))
print("salu/valu", round(g("SQ_INSTS_SALU", 0) / max(1, g("SQ_INSTS_VALU", 1)), 3))
PY
