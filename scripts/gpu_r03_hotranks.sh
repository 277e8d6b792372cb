#!/bin/bash
# Hot-rank split sweep (PILOSA_TOPN_HOT): row-major hot kernel vs the
# column-major slot histogram for the tail ranks, bench src mix per batch.
set -o pipefail
mkdir -p gpurun_out/r03_hotranks
for h in 1024 2048 4096 8192; do
  PILOSA_TOPN_HOT=$h timeout -k 10 300 python -u scripts/topn_kbench.py --reps 5 > gpurun_out/r03_hotranks/hot$h.log 2>&1 || { tail -c 2000 gpurun_out/r03_hotranks/hot$h.log; exit 1; }
  echo "hot=$h $(grep '^{' gpurun_out/r03_hotranks/hot$h.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["index_build_s"], d["mix"])')"
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_topn_exec.py tests/test_gpu_executor.py -k "topn or TopN or rank" > gpurun_out/r03_hotranks/pytest.log 2>&1 || { tail -c 4000 gpurun_out/r03_hotranks/pytest.log; exit 1; }
tail -1 gpurun_out/r03_hotranks/pytest.log
