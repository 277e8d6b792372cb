#!/bin/bash
# Wide-width executor + TopN suites (2^22 sub-shards), the TopN and write suites at 2^20.
set -o pipefail
O=gpurun_out/r04_d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topn_exec.py tests/test_gpu_write.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_topn_write.log 2>&1
rc=$?; tail -3 $O/pytest_topn_write.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests/test_gpu_shardwidth.py -m gpu -q -x --timeout 880 --timeout-method thread -k wide > $O/pytest_wide.log 2>&1
rc2=$?; tail -c 3000 $O/pytest_wide.log
exit $(( rc > rc2 ? rc : rc2 ))
