#!/bin/bash
# Kernel trace of executor-path src TopN requests on the headline index.
set -o pipefail
R=$PWD
mkdir -p gpurun_out/r03_topnprof2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_topnprof2 -o topn -- python3 $R/scripts/prof_topn_src.py > $R/gpurun_out/r03_topnprof2/run.log 2>&1 || { tail -c 3000 $R/gpurun_out/r03_topnprof2/run.log; exit 1; }
grep "src:" $R/gpurun_out/r03_topnprof2/run.log
f=$(find $R/gpurun_out/r03_topnprof2 -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:14]:
    print("%-70s calls=%5s avg_us=%9.1f pct=%s" % (r["Name"][:70], r["Calls"], float(r["AverageNs"]) / 1e3, r["Percentage"]))
PY
