timeout -k 10 300 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topn_exec.py 2>&1 | tail -15
