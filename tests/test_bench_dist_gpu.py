"""bench.py's real per-rank path at world_size 2 on the GPU.

The CPU tests (test_bench_dist.py) cover the launcher through `--mock`; these
run the code the driver's N-GPU bench runs -- rank_setup, one gvx.Context per
rank, the kernels on each rank's batch, barrier-bracketed max-over-ranks timing,
the results all-gather / the configs[4] track gather to rank 0 -- with both
ranks on the box's one GPU.  RCCL refuses two ranks on one device, so the
collectives go over gloo (host tensors, coll_device); on an 8-GPU node the same
code takes nccl with one GPU per rank."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_two_ranks(extra, timeout=100):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--backend", "gloo", "--no-cpu"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="2", MASTER_ADDR="127.0.0.1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    return json.loads(lines[0])


def test_batch_two_ranks_gather():
    """configs[1] batch at world 2 with the per-step results all-gather."""
    d = _run_two_ranks(["--pairs", "16", "--steps", "4", "--warmup", "2", "--no-pre", "--no-factors", "--gather",
                        "--no-sequence"])
    assert d["n_gpus"] == 2 and d["steps"] == 4 and d["scaling"] == "weak"
    assert abs(d["value"] - 2 * 16 * 4 / (d["ms_per_step"] * 4e-3)) < 1e-3 * d["value"]
    assert 0.5 < d["kept_fraction"] <= 1.0
    assert d["sequence"] is None


def test_default_line_sequence_two_ranks():
    """The default line's "sequence" sub-object at world 2:
    each rank replays its own configs[4] sequence inside the line's run, rank 0
    receives both ranks' per-frame tracks, and every record set matches its
    owner's digest."""
    d = _run_two_ranks(["--pairs", "16", "--steps", "4", "--warmup", "2", "--no-pre", "--no-factors",
                        "--seq-frames", "48"], timeout=160)
    s = d["sequence"]
    assert s["n_gpus"] == 2 and s["frames_per_rank"] == 48 and s["steps"] == 32  # warm-up 2 -> one K = 16 batch
    assert s["gathered_ranks"] == 2 and s["gather_check"] is True and s["dist_backend"] == "gloo"
    assert len(s["all_digests"]) == 2 and s["all_digests"][0] != s["all_digests"][1]  # distinct sequences
    assert abs(s["value"] - 2 * s["steps"] / (s["ms_per_step"] * s["steps"] * 1e-3)) < 1e-3 * s["value"]
    assert s["tracks_per_frame_mean"] > 75


def test_sequence_two_ranks_track_gather():
    """configs[4] at world 2: each rank replays its own sequence; rank 0 gets
    both ranks' per-frame tracks, its own intact."""
    d = _run_two_ranks(["--config", "5", "--frames", "40", "--warmup", "4"])
    assert d["n_gpus"] == 2 and d["warmup"] == 16 and d["steps"] == 24  # warm-up rounded to the K = 16 batch
    assert d["gathered_ranks"] == 2 and d["gather_check"] is True


def test_factors_two_ranks():
    """configs[3] factor batch at world 2 (max over ranks of the factor leg)."""
    d = _run_two_ranks(["--config", "4", "--steps", "3", "--warmup", "1"])
    assert d["n_gpus"] == 2
