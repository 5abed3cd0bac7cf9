"""bench.py contract on CPU/gloo: the reference-loop path prints one JSON line, and an
injected hang ends with an error JSON line naming the phase within the deadline
(the first 8-GPU driver run must always yield a record)."""
import json
import os
import subprocess
import sys
import time

import pytest

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _run(n, extra, env_extra=None, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    for k in ("PTDT_FAULT_RANK", "PTDT_FAULT_STEP", "PTDT_FAULT_MODE"):
        if env_extra is None or k not in env_extra:
            env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n),
           "--device", "cpu", "--engine", "reference", *extra]
    t0 = time.monotonic()
    p = subprocess.run(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    # the record may share a line with another rank's unterminated output: take it from '{"metric"'
    lines = [json.loads(l[l.index('{"metric"'):]) for l in p.stdout.splitlines() if '{"metric"' in l]
    return p, lines, time.monotonic() - t0


def test_bench_cpu_reference_line():
    p, lines, _ = _run(2, ["--steps", "64", "--warmup", "8"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["steps"] == 64 and rec["value"] > 0
    assert rec["config"]["global_batch"] == 64 and rec["config"]["parallelism"] == "dp2"
    assert rec["vs_cpu_probe"] is not None and "error" not in rec


def test_bench_deadline_on_injected_hang():
    deadline = 20
    p, lines, wall = _run(2, ["--steps", "200", "--warmup", "8", "--deadline", str(deadline)],
                          {"PTDT_FAULT_RANK": "1", "PTDT_FAULT_STEP": "3", "PTDT_FAULT_MODE": "hang"})
    assert p.returncode != 0
    assert len(lines) == 1, (p.stdout[-2000:], p.stderr[-2000:])
    rec = lines[0]
    assert rec["value"] is None and "deadline" in rec["error"]
    assert rec["phase"].startswith("headline")
    assert deadline <= rec["elapsed_s"] < deadline + 15
    assert wall < deadline + 90


def test_bench_cpu_8_ranks_reports_start_skew():
    """8 ranks (the driver's N = 8 shape) on gloo: the record carries the timed region's start skew
    and whole-node window, and the spin barrier released every rank (skew well under a millisecond)."""
    p, lines, _ = _run(8, ["--steps", "20", "--warmup", "5"], timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1
    tm = lines[0]["timing"]["headline"]
    assert tm["release"].startswith("spin barrier")
    assert len(tm["per_rank_elapsed_us"]) == 8
    # (8 spinning processes on this 8-CPU container: allow scheduler noise; on the GPU node it is ~us)
    assert 0.0 <= tm["start_skew_us"] < 20000.0, tm
    assert tm["window_us"] >= max(tm["per_rank_elapsed_us"]) - 1.0


def test_spin_barrier_releases_together(tmp_path):
    """utils/spin_barrier.py over 4 gloo ranks: no wait() returns before every rank arrived (a rank
    arriving 50 ms late holds the others), repeatedly."""
    from torch.multiprocessing import spawn

    from tests import _workers

    world = 4
    spawn(_workers.spin_barrier_check, args=(world, free_port(), str(tmp_path)), nprocs=world)
    import torch

    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt")) for r in range(world)]
    for rnd in range(3):
        arrive = max(r["arrive"][rnd] for r in res)
        for r in res:
            assert r["leave"][rnd] >= arrive  # released only after the last arrival
        assert max(r["leave"][rnd] for r in res) - arrive < 0.05  # and promptly


@pytest.mark.parametrize("failing_rank", [0, 2])
def test_spin_barrier_setup_failure_is_collective(tmp_path, failing_rank):
    """A rank that cannot create or map the shared page makes EVERY rank fall back to the collective
    barrier (create returns None everywhere) instead of leaving the others blocked."""
    import torch
    from torch.multiprocessing import spawn

    from tests import _workers

    world = 3
    spawn(_workers.spin_barrier_setup_failure, args=(world, free_port(), str(tmp_path), failing_rank), nprocs=world)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert all(r["none"] for r in res)
