#!/bin/bash
# Round 5, call I: cache-only TopN at full scale (954 shards, the wide
# distinct-call set) -- host profile of the request path and a kernel
# trace -- and the hot-rank TopN kernel counters (src TopN bound).
set -o pipefail
O=gpurun_out/r05_i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_topn_exec.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -c 5000 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python -u scripts/prof_topn_paths.py --cols 1000000000 --reqs 200 --paths local > $O/prof_topn_full.log 2>&1 || { tail -c 3000 $O/prof_topn_full.log; exit 1; }
grep -E "requests x|ms per" $O/prof_topn_full.log | head -5
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_topn -o topn -- python3 -u scripts/prof_topn_paths.py --cols 1000000000 --reqs 200 --paths local --top 5 > $O/prof_topn_trace.log 2>&1 || { tail -c 3000 $O/prof_topn_trace.log; exit 1; }
timeout -k 10 300 python3 -u scripts/topn_kbench.py --reps 1 > $O/topn_kbench.log 2>&1 || { tail -c 2000 $O/topn_kbench.log; exit 1; }
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $SET --kernel-include-regex "topn_hot_kernel" --output-format csv -d $O/hotpmc -o set$i -- python3 scripts/topn_kbench.py --reps 1 > $O/hotpmc_set$i.log 2>&1 || { tail -20 $O/hotpmc_set$i.log; exit 1; }
  echo "hot pmc pass $i done"
done
echo done
