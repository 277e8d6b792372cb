"""bench.py's --gpus contract (the driver runs ``bench.py --gpus N`` with or
without torch.distributed.run): a world size that disagrees with --gpus, or
more ranks than visible GPUs, fails fast with a non-zero exit instead of
timing one GPU and reporting it as N."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    env.pop("PILOSA_BENCH_REHEARSE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=300)


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


def test_more_gpus_than_visible_fails_before_launch():
    # this container has no GPU: --gpus 2 without a launcher must refuse, not run 1 rank
    r = _run(["--gpus", "2"], {})
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert "GPU(s) visible" in r.stderr or "cannot count GPUs from the KFD topology" in r.stderr


def test_kfd_gpu_count_reads_topology_without_hip(tmp_path, monkeypatch):
    """The launcher counts GPUs from the KFD topology (no HIP call before the
    ranks start): nodes with SIMDs are GPUs, the visibility lists cap them,
    and an unreadable topology is None (the launcher then refuses)."""
    sys.path.insert(0, ROOT)
    import bench
    for i, simds in enumerate([0, 1024, 1024, 0, 1024]):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 4\nsimd_count {simds}\nmax_waves_per_simd 8\n")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert bench.kfd_gpu_count(str(tmp_path)) == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.kfd_gpu_count(str(tmp_path)) == 1
    assert bench.kfd_gpu_count(str(tmp_path / "missing")) is None


def test_gpus_must_be_positive():
    r = _run(["--gpus", "0"], {})
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr
