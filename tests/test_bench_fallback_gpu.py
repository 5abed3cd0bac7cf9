"""bench.py's agreed engine chain on the GPU (utils/fallback.py): with the earlier engines failed by
injection, the fused engine's hipGraph path (capture + replay-vs-eager check), its eager path and
the native autograd engine each measure and report the path taken -- the code a multi-GPU node runs
when the in-kernel xGMI exchange or graph capture is unavailable there. The 2-rank shared-GPU case
fails the xGMI poll on one rank: every rank leaves the persistent engine, graph capture of the
host-staged all-reduce fails for real, and the eager fused engine measures."""
import json
import os
import subprocess
import sys

import pytest

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(args, inject, n=1, timeout=240):
    env = dict(os.environ, PTDT_BENCH_INJECT=inject)
    pre = ([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr",
            "127.0.0.1", "--master-port", str(free_port())] if n > 1 else [sys.executable])
    p = subprocess.run(pre + ["bench.py", "--gpus", str(n), *args], cwd=REPO, env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, timeout=timeout)
    lines = [json.loads(l[l.index('{"metric"'):]) for l in p.stdout.splitlines() if '{"metric"' in l]
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1
    return lines[0]


@pytest.mark.parametrize("inject,path,points", [
    ("stage:persistent", "fused_graph", ["stage:persistent"]),
    ("stage:persistent,graph_capture", "fused_eager", ["stage:persistent", "graph_capture"]),
    ("stage:persistent,graph_replay_check", "fused_eager", ["stage:persistent", "graph_replay_check"]),
    ("stage:persistent,stage:fused_graph,stage:fused_eager", "autograd",
     ["stage:persistent", "stage:fused_graph", "stage:fused_eager"]),
])
def test_bench_fallback_engines_measure(inject, path, points):
    rec = _bench(["--steps", "128", "--warmup", "16", "--no_ref", "--no_mlp_side"], inject)
    assert rec["engine_path"] == path and rec["config"]["engine"] == path
    assert [f["point"] for f in rec["fallback"]] == points
    assert rec["value"] > 0 and rec["n_gpus"] == 1


def test_bench_shared_gpu_poll_timeout_falls_back_together():
    rec = _bench(["--share_gpu", "--steps", "64", "--warmup", "8", "--no_mlp_side"], "xgmi_poll_timed@1", n=2)
    assert rec["engine_path"] == "fused_eager", rec.get("fallback")
    pts = [f["point"] for f in rec["fallback"]]
    assert pts == ["xgmi_poll_timed", "graph_capture"], rec["fallback"]
    assert set(rec["fallback"][0]["reasons"]) == {"1"}  # only rank 1 failed the poll; both moved on
    assert rec["value"] > 0 and rec["replicas_in_sync"]
