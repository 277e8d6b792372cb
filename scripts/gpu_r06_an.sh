#!/bin/bash
# Round 6, call AN: the driver's bench command with the 2000-request cache-only windows (no flags: N=1,
# every phase), then the world-size-1 RCCL mesh bench on the final code.
set -o pipefail
O=gpurun_out/r06_an
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -c 3000 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python3 -u bench.py > $O/bench.log 2> $O/bench.err || { tail -c 3000 $O/bench.err; exit 1; }
timeout -k 10 500 python3 -u bench.py --mesh --serve-seconds 0 --configs= > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 3000 $O/bench_mesh.err; exit 1; }
python3 - <<'PY'
import json
for n in ("bench", "bench_mesh"):
    d = json.loads([l for l in open(f"gpurun_out/r06_an/{n}.log") if l.startswith("{")][-1])
    e = d["extra"]; t = e.get("topn", {})
    print(n, d["value"], d["ms_per_step"], e.get("verified"), {k: (v.get("qps"), v.get("ms_per_request")) for k, v in t.items() if isinstance(v, dict) and "qps" in v})
    for k in ("config4_bsi", "config5_time_union", "serving"):
        if k in e: print("  ", k, json.dumps(e[k])[:600])
PY
echo done
