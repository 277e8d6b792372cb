#!/bin/bash
# GPU tests, 4-rank disk rehearsal of the N>1 bench path (device-tensor
# all-reduce), then a small 1-GPU bench with the serving + import phase.
set -o pipefail
mkdir -p gpurun_out/r03_check
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_check/pytest_gpu.log 2>&1 \
  || { tail -c 4000 gpurun_out/r03_check/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r03_check/pytest_gpu.log
NP=4 COLS=50000000 BATCH=1024 timeout -k 10 800 bash scripts/gpu_rehearse_disk.sh > gpurun_out/r03_check/rehearse.log 2>&1 \
  || { tail -c 3000 gpurun_out/r03_check/rehearse.log; exit 1; }
cat gpurun_out/r03_check/rehearse.log
cp gpurun_out/rehearse_disk*.log gpurun_out/r03_check/
timeout -k 10 400 python -u bench.py --cols 64000000 --steps 5 --warmup 2 --topn-batches 2 --configs none \
  --serve-seconds 3 --import-shards 32 > gpurun_out/r03_check/serve_small.log 2>&1 || { tail -c 3000 gpurun_out/r03_check/serve_small.log; exit 1; }
python - <<'PY'
import json
line = [l for l in open("gpurun_out/r03_check/serve_small.log") if l.startswith("{")][-1]
d = json.loads(line)
print(d["value"], json.dumps(d["extra"].get("serving"), indent=1))
PY
