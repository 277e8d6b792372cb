#!/usr/bin/env python3
"""Where a cache-only TopN request spends its time, single-rank executor vs
the world-size-1 RCCL mesh (the N-GPU product path), on a reduced copy of
the headline index (--cols, default 125M columns = 120 shards, one 8-GPU
rank's share).  Each path: warm-up, then --reqs requests of 16 distinct
calls timed, then the same under cProfile (top functions by own time).
Usage: python scripts/prof_topn_paths.py [--cols 125000000] [--reqs 300]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cols", type=int, default=125_000_000)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--reqs", type=int, default=300)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--topn-cache", type=int, default=50000)
    ap.add_argument("--paths", default="local,mesh")
    ap.add_argument("--top", type=int, default=35)
    ap.add_argument("--clients", default="1", help="comma list of request-thread counts to time (e.g. 1,2,3)")
    ap.add_argument("--wide", action="store_true", help="the bench's wide call set (n 1..1000, 72 thresholds)")
    args = ap.parse_args()
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": os.environ.get("MASTER_PORT", "29561"),
                       "RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    import math

    import torch

    import bench
    from pilosa_amd.executor import Executor
    from pilosa_amd.models.holder import Holder
    from pilosa_amd.ops.gpu_executor import GpuExecutor

    base = tempfile.mkdtemp(prefix="proftopn_")
    nshards = math.ceil(args.cols / bench.SHARD_WIDTH)
    bench._write_index(args, base, 0, nshards)
    holder = Holder(base, lazy_fragments=True).open()
    dev = torch.device("cuda", 0)
    gpu = GpuExecutor(holder, dev)
    ex = Executor(holder, gpu=gpu)
    gpu.executor = ex
    ex.strict_gpu = True
    shards = list(range(nshards))
    calls = bench._wide_topn_calls(16 * (args.reqs + 20)) if args.wide else \
        bench._distinct_topn_calls(16 * (args.reqs + 20))
    texts = [" ".join(calls[i * 16:(i + 1) * 16]) for i in range(args.reqs + 20)]

    def run_path(name):
        for t in texts[:20]:
            ex.execute("i", t, shards=shards)
        torch.cuda.synchronize()
        import threading
        for nc in [int(x) for x in args.clients.split(",") if x]:
            nxt = [20]
            lock = threading.Lock()

            def client():
                while True:
                    with lock:
                        i = nxt[0]
                        if i >= len(texts):
                            return
                        nxt[0] += 1
                    ex.execute("i", texts[i], shards=shards)
            t0 = time.perf_counter()
            ts = [threading.Thread(target=client) for _ in range(nc)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(f"{name}: {args.reqs} requests x 16 calls, {nc} request thread(s): "
                  f"{dt / args.reqs * 1000:.3f} ms/request, {16 * args.reqs / dt:.0f} q/s", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        for t in texts[20:]:
            ex.execute("i", t, shards=shards)
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(args.top)
        print(s.getvalue(), flush=True)
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(args.top)
        print(s.getvalue(), flush=True)

    paths = args.paths.split(",")
    if "local" in paths:
        run_path("local (single-rank executor)")
    if "mesh" in paths:
        from pilosa_amd.parallel.collectives import init
        from pilosa_amd.parallel.mesh import ShardMesh
        init("nccl", 0, timeout_s=60)
        mesh = ShardMesh(ex, block=nshards, device=dev, force=True)
        ex.mesh = mesh
        run_path("mesh (world-size-1 RCCL ShardMesh)")
        print("mesh data collectives:", mesh.comm.data_calls, "fused groups:", gpu.topn_mesh_fused, flush=True)
        mesh.stop()
        import torch.distributed as dist
        dist.destroy_process_group()
    ex.close()
    holder.close()
    import shutil
    shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
