"""Host C++ core under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference runs `go test -race` and a roaring fuzzer).
Builds pilosa_amd/native/selftest/roaring_selftest.cpp with the roaring core
and runs randomised ops against std::set (host code only: GPU sanitizers are
not available on this pool)."""
import os
import shutil
import subprocess
import tempfile

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(os.path.dirname(HERE), "pilosa_amd", "native")


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_roaring_core_asan_ubsan():
    out = os.path.join(tempfile.mkdtemp(), "roaring_selftest")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           "-fno-omit-frame-pointer", "-mpopcnt", "-mbmi2",
           os.path.join(NATIVE, "selftest", "roaring_selftest.cpp"), os.path.join(NATIVE, "roaring.cpp"), "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: tolerate libraries the environment preloads
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([out, "12"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "0 failures" in r.stderr


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
def test_roaring_core_threads_tsan():
    """Concurrent readers of shared bitmaps + per-thread writers under
    ThreadSanitizer, with the roaringstats counters compiled in (the host
    pool runs these ops with the GIL released)."""
    out = os.path.join(tempfile.mkdtemp(), "roaring_selftest_tsan")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-DPILOSA_ROARING_STATS", "-mpopcnt", "-mbmi2",
           "-pthread", os.path.join(NATIVE, "selftest", "roaring_selftest.cpp"), os.path.join(NATIVE, "roaring.cpp"),
           "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([out, "6", "threads"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "threads: 0 failures" in r.stderr
