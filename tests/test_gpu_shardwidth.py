"""Device arenas at shard widths other than the device shard's 2^20 columns
(reference shardwidth/16.go..32.go): narrower (2^16, 2^18): the GPU executor's
differential suite and the executor-path TopN suite run unchanged at that
width in a fresh interpreter (the width is fixed per process, like the
reference's build tag), every answer compared with the host executor.
Wider (2^22, the reference CI's SHARD_WIDTH=22): every shard is 4 device
sub-shards and the executor and TopN suites run unchanged (rank caches stay
per fragment with counts summed over its sub-shards; src TopN runs on the
slot index built per sub-shard, its histograms summed per fragment, and
tests/test_gpu_topn_exec.py asserts the slot index answered).
Shift carries across the sub-shards of a wide shard on the device; at the
narrow widths a shard's spill starts at its own 2^e columns (row_kernels.hip
shift_dense row_words), so the Shift tests run there too and assert device
launches."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
@pytest.mark.parametrize("exp", [16, 18])
def test_gpu_suites_at_narrow_width(exp):
    env = dict(os.environ, PILOSA_SHARD_WIDTH=str(exp))
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        "--timeout", "300", "--timeout-method", "thread",
                        "tests/test_gpu_executor.py", "tests/test_gpu_topn_exec.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "skipped" not in r.stdout.splitlines()[-1], r.stdout[-1000:]


@pytest.mark.timeout(900)
def test_gpu_executor_suite_at_wide_width():
    """Shift included: the device carries across the 4 sub-shards of a 2^22
    shard, and its test asserts a device launch (no host fallback)."""
    env = dict(os.environ, PILOSA_SHARD_WIDTH="22")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        "--timeout", "300", "--timeout-method", "thread",
                        "tests/test_gpu_executor.py", "tests/test_gpu_topn_exec.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=850)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    last = r.stdout.splitlines()[-1]
    # skips allowed: the two engine-level ops/topn.py tests (per arena shard)
    assert " passed" in last and ("skipped" not in last or "2 skipped" in last), r.stdout[-1000:]


@pytest.mark.timeout(600)
def test_gpu_topn_suites_with_wide_lane_owned_rows():
    """The hot-rank TopN kernel with lane-owned containers up to 1023 values
    (PILOSA_TOPN_SMALL_N=1023: carry-save planes counted every 240 values) answers
    the slot-index and executor TopN suites exactly."""
    env = dict(os.environ, PILOSA_TOPN_SMALL_N="1023")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "gpu",
                        "--timeout", "300", "--timeout-method", "thread", "-k", "slot_index or topn or TopN",
                        "tests/test_gpu_executor.py", "tests/test_gpu_topn_exec.py"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=580)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert " passed" in r.stdout.splitlines()[-1], r.stdout[-1000:]
