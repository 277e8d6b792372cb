#!/bin/bash
# TopN GPU suite (lane pool concurrency test included).
set -o pipefail
O=gpurun_out/r04_m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topn_exec.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 3000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
