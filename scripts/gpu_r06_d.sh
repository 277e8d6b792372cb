#!/bin/bash
# Round 6, call D: pair kernel bank conflicts. Lane-rotated chunks (variant 50)
# vs the shipped v6: kernel time (kbench, 4096-query batch, full 954-shard
# arena) and LDS counters, one variant per rocprofv3 pass.
set -o pipefail
R=$PWD
O=$R/gpurun_out/r06_d
mkdir -p $O
timeout -k 10 300 python3 -u scripts/kbench.py --batch 4096 --reps 10 --cq 64 --no-tile --variants 50,6,50 > $O/kbench.log 2>&1 || { tail -30 $O/kbench.log; exit 1; }
grep -v "^{" $O/kbench.log
cd /tmp && export TMPDIR=/tmp
for V in 6 50; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU --kernel-include-regex "and2_pairs_v6" --output-format csv -d $O/pmc -o v$V -- python3 $R/scripts/kbench.py --reps 1 --cq "" --variants $V@64 --no-tile --batch 4096 > $O/pmc_v$V.log 2>&1 || { tail -20 $O/pmc_v$V.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r06_d/pmc/v*_counter_collection.csv")):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        d[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f.split("/")[-1], {k: f"{v:.4g}" for k, v in sorted(d.items())})
    if d["SQ_LDS_IDX_ACTIVE"]:
        print("  lds_bank_conflict/active", round(d["SQ_LDS_BANK_CONFLICT"] / d["SQ_LDS_IDX_ACTIVE"], 3))
PY
echo done
