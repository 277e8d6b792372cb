"""Host C++ core under AddressSanitizer + UndefinedBehaviorSanitizer
(the reference runs `go test -race` and a roaring fuzzer).
Builds pilosa_amd/native/selftest/roaring_selftest.cpp with the roaring core
and runs randomised ops against std::set (host code only: GPU sanitizers are
not available on this pool)."""
import os
import shutil
import subprocess
import sys
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


# ------------------------------------------------------------------ the other
# native modules: each is built with the sanitizer into a scratch dir and
# driven from a Python interpreter with the sanitizer runtime preloaded
# (pilosa_amd/native/selftest/san_driver.py: concurrent use plus malformed,
# truncated and mutated input; the PQL parser's nesting bound came out of the
# ASan stack-overflow report of this driver)
DRIVER = os.path.join(NATIVE, "selftest", "san_driver.py")
MODULES = {"httpd": "_httpd", "translate": "_translate", "arena": "_roaring", "pql": "_pql"}


def _runtime(lib):
    p = subprocess.run(["g++", f"-print-file-name={lib}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.slow
@pytest.mark.skipif(shutil.which("g++") is None, reason="no host compiler")
@pytest.mark.parametrize("mode", sorted(MODULES))
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_native_module_sanitized(mode, san):
    from pilosa_amd.native.build import build_sanitized
    rt = _runtime("libtsan.so" if san == "thread" else "libasan.so")
    if rt is None:
        pytest.skip("sanitizer runtime not installed")
    d = tempfile.mkdtemp()
    try:
        build_sanitized(MODULES[mode], san, d)
        env = dict(os.environ, PYTHONPATH=os.path.dirname(NATIVE.rstrip("/")).rsplit(os.sep, 1)[0])
        if san == "thread":
            env.update(LD_PRELOAD=rt, TSAN_OPTIONS="halt_on_error=1:exitcode=66:suppressions="
                       + os.path.join(NATIVE, "selftest", "tsan.supp"))
        else:
            stdcxx = _runtime("libstdc++.so")
            env.update(LD_PRELOAD=rt + (":" + stdcxx if stdcxx else ""),
                       ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
                       UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
        r = subprocess.run([sys.executable, DRIVER, d, mode, "5"], capture_output=True, text=True, timeout=600,
                           env=env, cwd=d)
        assert r.returncode == 0, r.stderr[-6000:]
        assert f"{mode}: ok" in r.stderr
    finally:
        shutil.rmtree(d, ignore_errors=True)
