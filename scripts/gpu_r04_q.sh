#!/bin/bash
# TopN / executor / shard-width GPU suites at the current defaults.
set -o pipefail
O=gpurun_out/r04_q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_executor.py tests/test_gpu_shardwidth.py -m gpu -q -x --timeout 800 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 3000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
