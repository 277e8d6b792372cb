#!/bin/bash
# kernel trace of the Count(Intersect) batch harness (scripts/kbench.py, one config)
set -o pipefail
R=$PWD
mkdir -p $R/gpurun_out/kprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kprof -o ${TAG:-k} -- \
  python3 $R/scripts/kbench.py --batch ${BATCH:-4096} --cq 0 --reps 3 ${KB_ARGS} > $R/gpurun_out/kprof_${TAG:-k}.log 2>&1 || { tail -30 $R/gpurun_out/kprof_${TAG:-k}.log; exit 1; }
head -8 $R/gpurun_out/kprof/${TAG:-k}_kernel_stats.csv | cut -c 1-150
