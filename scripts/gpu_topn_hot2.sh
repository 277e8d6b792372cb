#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "slot_index" \
  > gpurun_out/pt_topn.log 2>&1 || { tail -30 gpurun_out/pt_topn.log; exit 1; }
tail -1 gpurun_out/pt_topn.log
timeout -k 10 200 python -u scripts/topn_hot_probe.py --shards 128 > gpurun_out/tpmc_probe.log 2>&1 || { tail -20 gpurun_out/tpmc_probe.log; exit 1; }
tail -1 gpurun_out/tpmc_probe.log
timeout -k 10 200 python -u scripts/topn_hot_probe.py --shards 954 --src 0 > gpurun_out/tpmc_probe.log 2>&1 || { tail -20 gpurun_out/tpmc_probe.log; exit 1; }
tail -1 gpurun_out/tpmc_probe.log
