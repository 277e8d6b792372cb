"""Runtime profiles behind ``/debug/pprof/`` (reference: net/http/pprof
mounted at http/handler.go:280).

Go's pprof endpoints map onto what a Python + native runtime can observe:

* ``profile?seconds=N`` -- a statistical CPU profile: every thread's stack is
  sampled ``hz`` times a second for N seconds and returned in the folded
  ("collapsed stack") format that flamegraph.pl / speedscope read, hottest
  stacks first.  Native frames (the C++ roaring core, HIP launches) show up
  as the Python frame that called into them.
* ``goroutine`` -- a dump of every thread's current stack (debug=1: grouped).
* ``heap`` -- tracemalloc top allocation sites (``?start=1`` starts tracing,
  ``?stop=1`` stops it) plus live object counts by type from the collector.
* ``threadcreate`` -- live threads.
* ``cmdline`` -- the process command line.
* ``gpu`` -- caching-allocator statistics of every visible GPU.
"""
from __future__ import annotations

import collections
import gc
import sys
import threading
import time
import traceback
from typing import Dict, List

INDEX = ["profile", "goroutine", "heap", "threadcreate", "cmdline", "gpu"]


def _frame_label(fr) -> str:
    co = fr.f_code
    return f"{co.co_name} ({co.co_filename.rsplit('/', 1)[-1]}:{fr.f_lineno})"


def _stack(fr) -> List[str]:
    out = []
    while fr is not None:
        out.append(_frame_label(fr))
        fr = fr.f_back
    out.reverse()
    return out


def cpu_profile(seconds: float = 30.0, hz: int = 100) -> str:
    """Folded stacks "thread;outer;...;inner count" over ``seconds``."""
    seconds = max(0.05, min(float(seconds), 300.0))
    hz = max(1, min(int(hz), 1000))
    me = threading.get_ident()
    names = {t.ident: t.name for t in threading.enumerate()}
    counts: Dict[str, int] = collections.Counter()
    deadline = time.perf_counter() + seconds
    period = 1.0 / hz
    samples = 0
    while time.perf_counter() < deadline:
        for tid, fr in sys._current_frames().items():
            if tid == me:
                continue
            counts[";".join([names.get(tid, str(tid))] + _stack(fr))] += 1
        samples += 1
        time.sleep(period)
    lines = [f"# pilosa_amd cpu profile: {samples} samples at {hz} Hz over {seconds:.2f} s (folded stacks)"]
    lines += [f"{k} {v}" for k, v in sorted(counts.items(), key=lambda kv: -kv[1])]
    return "\n".join(lines) + "\n"


def goroutine(debug: int = 0) -> str:
    names = {t.ident: t.name for t in threading.enumerate()}
    frames = sys._current_frames()
    if debug >= 1:   # identical stacks grouped, like goroutine?debug=1
        groups: Dict[str, List[str]] = collections.defaultdict(list)
        for tid, fr in frames.items():
            groups["".join(traceback.format_stack(fr))].append(names.get(tid, str(tid)))
        out = [f"threads: {len(frames)}"]
        for st, who in sorted(groups.items(), key=lambda kv: -len(kv[1])):
            out.append(f"\n{len(who)} @ {', '.join(sorted(who))}\n{st}")
        return "\n".join(out)
    return "\n".join(f"--- thread {names.get(tid, tid)} ({tid})\n" + "".join(traceback.format_stack(fr))
                     for tid, fr in frames.items())


def heap(start: bool = False, stop: bool = False, top: int = 50) -> str:
    import tracemalloc
    if start and not tracemalloc.is_tracing():
        tracemalloc.start(16)
    out = []
    if tracemalloc.is_tracing():
        snap = tracemalloc.take_snapshot()
        stats = snap.statistics("traceback")
        cur, peak = tracemalloc.get_traced_memory()
        out.append(f"# tracemalloc: current {cur} B, peak {peak} B, top {top} sites")
        for st in stats[:top]:
            out.append(f"{st.size} B in {st.count} blocks")
            out.extend("    " + ln for ln in st.traceback.format())
    else:
        out.append("# tracemalloc is off (GET /debug/pprof/heap?start=1 to start tracing)")
    if stop and tracemalloc.is_tracing():
        tracemalloc.stop()
    by_type = collections.Counter(type(o).__name__ for o in gc.get_objects())
    out.append(f"\n# live objects by type (gc), {sum(by_type.values())} total")
    out.extend(f"{n} {t}" for t, n in by_type.most_common(top))
    return "\n".join(out) + "\n"


def threadcreate() -> str:
    ts = threading.enumerate()
    return f"threads: {len(ts)}\n" + "\n".join(f"{t.ident} {t.name} daemon={t.daemon}" for t in ts) + "\n"


def cmdline() -> str:
    return "\x00".join(sys.argv)


def gpu() -> str:
    try:
        import torch
        if not torch.cuda.is_available():
            return "no GPU visible\n"
        out = []
        for d in range(torch.cuda.device_count()):
            s = torch.cuda.memory_stats(d)
            out.append(f"device {d}: allocated {s.get('allocated_bytes.all.current', 0)} B, "
                       f"reserved {s.get('reserved_bytes.all.current', 0)} B, "
                       f"peak {s.get('allocated_bytes.all.peak', 0)} B, "
                       f"alloc retries {s.get('num_alloc_retries', 0)}")
        return "\n".join(out) + "\n"
    except Exception as e:  # noqa: BLE001
        return f"gpu stats unavailable: {e}\n"


def index_page() -> str:
    return "/debug/pprof/\n\nprofiles:\n" + "\n".join(f"  {p}" for p in INDEX) + "\n"


def render(rest: str, query: Dict[str, str]) -> str:
    """Dispatch ``/debug/pprof/<rest>``; KeyError for unknown profiles."""
    name = rest.strip("/")
    if name == "":
        return index_page()
    if name == "profile":
        return cpu_profile(float(query.get("seconds", 30)), int(query.get("hz", 100)))
    if name == "goroutine":
        return goroutine(int(query.get("debug", 0)))
    if name in ("heap", "allocs"):
        return heap(query.get("start") in ("1", "true"), query.get("stop") in ("1", "true"))
    if name == "threadcreate":
        return threadcreate()
    if name == "cmdline":
        return cmdline()
    if name == "gpu":
        return gpu()
    raise KeyError(name)
