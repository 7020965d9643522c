"""bench.py's multi-process contract on CPU (gloo, world_size 2): launched like
the driver launches it (torch.distributed.run, 127.0.0.1), rank 0 prints one
JSON line, the timed region is max-over-ranks, value is the whole-job
aggregate (weak scaling)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_mock_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--mock", "--backend", "gloo", "--gpus", "2", "--steps", "20", "--warmup", "2", "--pairs", "8"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 20 and d["scaling"] == "weak"
    # rank 1 sleeps 4 ms per step: the max over ranks must be >= 20 * 4 ms
    assert d["elapsed_s"] >= 0.08
    assert abs(d["value"] - 2 * 8 * 20 / d["elapsed_s"]) < 1e-6 * d["value"]
    # the clock warm-up side legs run before the headline on EVERY rank at N > 1,
    # as at N = 1
    assert d["side_legs_before_headline"] == ["lk_accum", "preprocess", "settle"]
    assert d["side_legs_before_headline_ranks"] == 2


def test_bench_mock_sequence_gather_gloo():
    """configs[4]'s exchange: per-frame tracks of every rank reach rank 0 intact."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--mock", "--config", "5", "--backend", "gloo", "--gpus", "2", "--steps", "4", "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    assert json.loads(lines[0])["gathered_ok"] is True


def test_bench_spawns_ranks_itself():
    """`bench.py --gpus 2` with no launcher starts its own 2 ranks (the driver's
    N-GPU runs and a user's plain invocation give the same job)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mock", "--backend", "gloo", "--gpus", "2",
           "--steps", "10", "--warmup", "1", "--pairs", "4"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    assert json.loads(lines[0])["n_gpus"] == 2


def test_bench_rejects_world_mismatch():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--mock", "--gpus", "2"]
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert out.returncode != 0 and "WORLD_SIZE" in out.stderr


def test_bench_mock_default_line_sequence_gloo():
    """The default line's "sequence" sub-object at world 2:
    the configs[4] exchange -- every rank's records gathered to rank 0, checked
    against the all-gathered per-rank digests -- aggregated over both ranks."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--mock", "--backend", "gloo", "--gpus", "2", "--steps", "4", "--warmup", "1", "--pairs", "8"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    s = json.loads(lines[0])["sequence"]
    assert s["n_gpus"] == 2 and s["gathered_ranks"] == 2 and s["gather_check"] is True
    assert s["dist_backend"] == "gloo" and len(s["all_digests"]) == 2
    assert s["all_digests"][0] != s["all_digests"][1]
    assert s["value"] > 0 and s["scaling"] == "weak"
