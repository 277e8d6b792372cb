#!/usr/bin/env python3
"""BASELINE configs 4 / 5 (bench.bench_configs_disk) under cProfile: where
a BSI Sum / range / Min / Max request (or a time-union batch) spends its
host time next to the kernels (run it under rocprofv3 --kernel-trace
--stats for the device side).  Prints the bench's JSON and the top
functions by own and cumulative time.
Usage: python scripts/prof_configs.py [--which 4] [--reps 20]"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", default="4")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cols", type=int, default=1_000_000_000)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--no-profile", action="store_true", help="no cProfile (under rocprofv3)")
    a = ap.parse_args()
    import torch

    import bench
    args = argparse.Namespace(cols=a.cols, rows=a.rows, threads=a.threads, data_dir=None, keep_data=False,
                              config_reps=a.reps)
    dev = torch.device("cuda", 0)
    pr = cProfile.Profile()
    if not a.no_profile:
        pr.enable()
    res = bench.bench_configs_disk(args, 1, 0, dev, a.which)
    pr.disable()
    print(json.dumps(res), flush=True)
    if a.no_profile:
        return
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
