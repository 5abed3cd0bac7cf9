"""Agreed engine fallback (utils/fallback.py, bench.py's chain) on CPU/gloo: a failure injected on
ONE rank at any decision point -- xGMI init, an xGMI poll timeout, graph capture, a replay that
differs from its eager run, an unexpected local exception -- moves EVERY rank to the same next
engine, and bench.py still prints exactly one valid JSON line naming the path and the reasons
(the first 8-GPU driver run must yield a number whatever happens)."""
import json
import os
import subprocess
import sys

import pytest
import torch
from torch.multiprocessing import spawn

from pytorch_distributed_training_tutorials_amd.parallel.env import free_port

from . import _workers

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _chain(tmp_path, world, inject):
    spawn(_workers.fallback_chain, args=(world, free_port(), str(tmp_path), inject), nprocs=world)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(world)]
    for r in res[1:]:  # every rank took the same path, through the same decision points
        assert r == res[0]
    return res[0]


@pytest.mark.parametrize("inject,path,point", [
    ("", "persistent", None),
    ("xgmi_init@1", "fused_graph", "xgmi_init"),
    ("xgmi_poll_timed@2", "fused_graph", "xgmi_poll_timed"),
    ("xgmi_poll_warmup@0,graph_capture@1", "fused_eager", "graph_capture"),
    ("xgmi_init@2,replay_diff", "fused_eager", "graph_replay_check"),
    ("xgmi_init@1,graph_capture@2,crash@1", "reference", "stage:fused_eager"),
    ("stage:persistent@0", "fused_graph", "stage:persistent"),
    ("stage:fused_graph@2,xgmi_poll_warmup@1", "fused_eager", "stage:fused_graph"),
])
def test_chain_agreed_across_ranks(tmp_path, inject, path, point):
    out = _chain(tmp_path, 3, inject)
    assert out["name"] == path
    assert out["res"] == f"{path.replace('_', '-')}-result"
    if point is None:
        assert out["failures"] == []
    else:
        assert out["failures"][-1]["point"] == point
        assert all(f["reasons"] for f in out["failures"])
        toks = dict(t.split("@") for t in inject.split(",") if "@" in t)
        for f in out["failures"]:  # an injected point names only the injected rank (the others moved on)
            if f["point"] in toks:
                assert set(f["reasons"]) == {toks[f["point"]]}, out["failures"]


def test_chain_every_stage_failed(tmp_path):
    out = _chain(tmp_path, 2, "stage:persistent@1,stage:fused_graph@0,stage:fused_eager@1,stage:reference@0")
    assert out["name"] is None and "every stage" in out["error"]


def test_chain_desync_is_detected_by_every_rank(tmp_path):
    """A rank leaving a stage by a local exception before a decision point the others reach: the
    named decision points disagree and EVERY rank stops (no wrong pairing of collectives)."""
    spawn(_workers.fallback_chain, args=(3, free_port(), str(tmp_path), "xgmi_init@0,early@1"), nprocs=3)
    res = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(3)]
    assert all(r == {"name": None, "desync": True} for r in res)


def _bench(n, extra, env_extra=None, timeout=300):
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n),
           "--device", "cpu", *extra]
    p = subprocess.run(cmd, cwd=REPO, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    lines = [json.loads(l[l.index('{"metric"'):]) for l in p.stdout.splitlines() if '{"metric"' in l]
    return p, lines


@pytest.mark.slow
def test_bench_chain_reaches_a_number_on_cpu():
    """--engine persistent on CPU: the GPU engines fail their agreed 'device' point on every rank and
    the chain ends at the stock loop, which measures; one JSON line with the whole path."""
    p, lines = _bench(2, ["--engine", "persistent", "--steps", "32", "--warmup", "4", "--no_ref"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert len(lines) == 1
    rec = lines[0]
    assert rec["value"] > 0 and rec["engine_path"] == "reference" and rec["config"]["engine"] == "reference"
    assert [f["stage"] for f in rec["fallback"]] == ["persistent", "fused_graph", "fused_eager", "autograd"]
    assert all(f["point"] == "device" and set(f["reasons"]) == {"0", "1"} for f in rec["fallback"])


@pytest.mark.slow
def test_bench_chain_all_failed_prints_error_line():
    p, lines = _bench(2, ["--engine", "autograd", "--steps", "16", "--warmup", "2", "--no_ref"],
                      {"PTDT_BENCH_INJECT": "stage:reference@1"})
    assert p.returncode != 0
    assert len(lines) == 1
    assert lines[0]["value"] is None and "every engine failed" in lines[0]["error"]
