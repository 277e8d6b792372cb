#!/bin/bash
# End-to-end HTTP serving on the config-2 index (1B cols x 1M rows as
# Pilosa-format fragment files, scripts/bench_server.py): native front end
# (native/httpd.cpp + Count group commit) vs the stdlib ThreadingHTTPServer,
# 128 keep-alive connections from the native load client.
set -o pipefail
mkdir -p gpurun_out
D=${TMPDIR:-/tmp}/pilosa_serve_data
for srvmode in 1 0; do
  PILOSA_NATIVE_HTTP=$srvmode timeout -k 10 400 python -u scripts/bench_server.py --data-dir $D --cols ${COLS:-1000000000} \
    --conns ${CONNS:-128} --seconds ${SECS:-10} > gpurun_out/serving_native$srvmode.log 2>&1 \
    || { tail -20 gpurun_out/serving_native$srvmode.log; exit 1; }
  tail -1 gpurun_out/serving_native$srvmode.log
done
