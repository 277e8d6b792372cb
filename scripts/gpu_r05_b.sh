#!/bin/bash
# Round 5, call B: (1) mesh GPU tests (RCCL world 1 + gloo 2-rank) with the
# node-wide fused cache-only TopN; (2) pair-kernel cost attribution: v6 vs its
# DBG variants 31-35 (skeleton / no wave_sum / no staging / no counting /
# skeleton without B loads); (3) PMC passes over v6 and the skeleton;
# (4) bench --gpus 1 --mesh and the 4-rank rehearsal vs 1 rank.
set -o pipefail
R=$PWD
O=gpurun_out/r05_b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl_mesh.py tests/test_gpu_mesh.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -c 6000 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
timeout -k 10 600 python -u scripts/kbench.py --batch 4096 --reps 5 --cq 64 --no-tile --variants 31,32,33,34,35 > $O/kbench_attr.log 2>&1 || { tail -c 3000 $O/kbench_attr.log; exit 1; }
grep -v "^{" $O/kbench_attr.log | tail -8
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $SET --kernel-include-regex "and2_pairs_v6" --output-format csv -d $R/$O/pmc -o set$i -- python3 $R/scripts/kbench.py --reps 1 --cq 64 --no-tile --variants 31 --batch 4096 > $R/$O/pmc_set$i.log 2>&1 || { tail -20 $R/$O/pmc_set$i.log; exit 1; }
  echo "pmc pass $i done"
done
cd $R
python3 - <<'PY' > gpurun_out/r05_b/pmc_summary.txt
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob("gpurun_out/r05_b/pmc/**/set*_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        k = "DBG1 skeleton" if ", 1>" in k else "v6 shipped" if "and2_pairs_v6" in k else k[:60]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:28s} {v:.4g}")
PY
cat gpurun_out/r05_b/pmc_summary.txt
ARGS="--steps 20 --warmup 5 --configs= --serve-seconds 0 --topn-batches 20 --topn-pairs-batches 0"
timeout -k 10 900 python -u bench.py --gpus 1 --mesh $ARGS > $O/bench_mesh.log 2> $O/bench_mesh.err || { tail -c 5000 $O/bench_mesh.err; exit 1; }
RARGS="--cols 125000000 --batch 1024 --steps 5 --warmup 2 --configs= --serve-seconds 0 --topn-batches 10 --topn-pairs-batches 0 --clients 3"
timeout -k 10 600 env PILOSA_BENCH_REHEARSE=1 python -u bench.py --gpus 4 $RARGS > $O/bench4.log 2> $O/bench4.err || { tail -c 5000 $O/bench4.err; exit 1; }
python - <<'PY'
import json
for n in ("_mesh", "4"):
    d = json.loads([l for l in open(f"gpurun_out/r05_b/bench{n}.log") if l.startswith("{")][-1])
    e = d["extra"]
    t = e.get("topn", {})
    print(n, "n_gpus", d["n_gpus"], "value", d["value"], "ms", d["ms_per_step"], "verified", d["verified"],
          "backend", e.get("backend"), "world", e.get("world_size"), "inflight", e.get("mesh_max_in_flight"))
    print("  topn cache", {k: t.get("cache", {}).get(k) for k in ("qps", "ms_per_request", "max_in_flight")},
          "src", {k: t.get("src", {}).get(k) for k in ("qps", "ms_per_request")}, "verify", t.get("verify"))
PY
