#!/bin/bash
# BSI kernels: GPU tests, then config 4 timings for both sum variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "bsi or BSI or Sum or sum" --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_bsi.log 2>&1 || { tail -30 gpurun_out/pytest_bsi.log; exit 1; }
tail -2 gpurun_out/pytest_bsi.log
for v in ${VARIANTS:-0 1}; do
  PILOSA_BSI_SUM_VARIANT=$v timeout -k 10 300 python -u scripts/bench_configs.py --only 4 > gpurun_out/bsi_v$v.log 2>&1 \
    || { tail -20 gpurun_out/bsi_v$v.log; exit 1; }
  echo "variant $v"; tail -1 gpurun_out/bsi_v$v.log
done
