#!/bin/bash
# Round 6, call M: src TopN batch breakdown on the headline arena
# (topn_kbench: materialize / hot-rank kernel / phase 1 / candidates / phase
# 2), then PMC passes over the hot-rank kernel (occupancy, LDS, VALU, waits).
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_m
mkdir -p $O
timeout -k 10 400 python3 -u scripts/topn_kbench.py --reps 5 > $O/topn_kbench.log 2>&1 || { tail -30 $O/topn_kbench.log; exit 1; }
grep "^{" $O/topn_kbench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d.get('mix')), json.dumps(d.get('classes')))"
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
for f in sorted(glob.glob("gpurun_out/r06_m/pmc/set*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k, {c: f"{v:.4g}" for c, v in sorted(d.items())})
    g = lambda n: d.get(n, 0.0)
    if g("SQ_LDS_IDX_ACTIVE"): print("  lds_conflict/active", round(g("SQ_LDS_BANK_CONFLICT") / g("SQ_LDS_IDX_ACTIVE"), 3))
    if g("SQ_WAVE_CYCLES"): print("  wait_any/wave_cycles", round(g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES"), 3), "busy/gui", round(g("SQ_BUSY_CYCLES") / max(g("GRBM_GUI_ACTIVE"), 1), 3))
    if g("TCC_HIT_sum") + g("TCC_MISS_sum"): print("  l2_hit", round(g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")), 3))
PY
timeout -k 10 400 env PILOSA_BENCH_TOPN_PROFILE=$O/plain_topn.folded PILOSA_BENCH_CPROFILE=$O/plain_topn_cprofile.txt python3 -u bench.py --serve-seconds 0 --configs= --steps 3 --warmup 1 --topn-src-batches 40 > $O/bench_prof.log 2> $O/bench_prof.err || { tail -c 3000 $O/bench_prof.err; exit 1; }
head -40 $O/plain_topn_cprofile.txt
echo done
