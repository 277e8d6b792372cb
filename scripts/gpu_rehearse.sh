#!/bin/bash
# NP-rank (default 2) rehearsal of the N-GPU bench path on a 1-GPU box (gloo collectives
# through host copies), then a kernel-trace profile of the TopN paths.
set -o pipefail
mkdir -p gpurun_out/prof
NP=${NP:-2}
PILOSA_BENCH_REHEARSE=1 timeout -k 10 ${RTIMEOUT:-300} python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $NP --steps 3 --warmup 1 --cols ${COLS:-100000000} \
  --batch ${BATCH:-1024} > gpurun_out/rehearse$NP.log 2>&1 || { tail -c 2000 gpurun_out/rehearse$NP.log; exit 1; }
tail -c 1500 gpurun_out/rehearse$NP.log
[ -n "$PROFILE" ] || exit 0
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o ${TAG:-topn} -- \
  python3 $R/bench.py --steps 2 --warmup 1 --batch 256 --topn-batches 3 --topn-pairs-batches 0 \
  > $R/gpurun_out/prof_${TAG:-topn}.log 2>&1 || { tail -30 $R/gpurun_out/prof_${TAG:-topn}.log; exit 1; }
echo PROFILE_DONE
