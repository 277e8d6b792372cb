#!/bin/bash
# Multi-rank rehearsal of the disk-mode bench on a 1-GPU box (gloo through host
# copies): NP=1 and NP=4 on the same config must report the same mean count.
set -o pipefail
mkdir -p gpurun_out
A="--steps 3 --warmup 1 --cols ${COLS:-100000000} --batch ${BATCH:-1024} --topn-batches 1 --topn-pairs-batches 1"
timeout -k 10 300 python -u bench.py $A > gpurun_out/rehearse_disk1.log 2>&1 || { tail -c 2000 gpurun_out/rehearse_disk1.log; exit 1; }
PILOSA_BENCH_REHEARSE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-4} \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus ${NP:-4} $A > gpurun_out/rehearse_disk${NP:-4}.log 2>&1 \
  || { tail -c 3000 gpurun_out/rehearse_disk${NP:-4}.log; exit 1; }
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/rehearse_disk*.log")):
    line = [l for l in open(f) if l.startswith("{")][-1]
    d = json.loads(line)
    t = d["extra"].get("topn", {})
    print(f, d["n_gpus"], d["value"], d["verified"], d["extra"]["mean_count"],
          t.get("cache", {}).get("sample_top3"), t.get("src", {}).get("sample_top3"), t.get("src_paths_agree"), t.get("cache_paths_agree"))
PY
