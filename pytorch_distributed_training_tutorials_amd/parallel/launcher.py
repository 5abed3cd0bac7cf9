"""Process launchers.

* :func:`spawn` -- ``torch.multiprocessing.spawn`` equivalent (ddp_gpus.py:104-105):
  one fresh ``spawn``-context process per rank, ``fn(rank, *args)``; the parent
  joins, and the first failing child tears the whole group down (no orphaned
  ranks blocked in a collective) and its exception/exit code is re-raised.
* :func:`launch` / ``python -m pytorch_distributed_training_tutorials_amd.launch``
  -- a torchrun-compatible launcher for one node: exports the elastic env
  contract (``RANK, LOCAL_RANK, WORLD_SIZE, LOCAL_WORLD_SIZE, GROUP_RANK,
  ROLE_RANK, MASTER_ADDR, MASTER_PORT, TORCHELASTIC_RESTART_COUNT,
  TORCHELASTIC_MAX_RESTARTS, TORCHELASTIC_RUN_ID``), sets ``OMP_NUM_THREADS=1``
  with torchrun's warning when nproc > 1, monitors the workers, kills the
  group when one fails, and restarts the whole group up to ``--max-restarts``
  times. ``--nnodes/--node-rank`` give the fake multi-node layout of SURVEY §4
  item 5 (ranks = node_rank * nproc + local_rank).
"""
from __future__ import annotations

import argparse
import multiprocessing as mp
import os
import signal
import subprocess
import sys
import time
import traceback
import uuid


class ProcessRaisedException(RuntimeError):
    pass


def _spawn_entry(fn, rank, args, err_q):
    try:
        fn(rank, *args)
    except BaseException:  # noqa: BLE001
        err_q.put((rank, traceback.format_exc()))
        sys.exit(1)


def spawn(fn, args=(), nprocs: int = 1, join: bool = True, poll_s: float = 0.1):
    ctx = mp.get_context("spawn")
    err_q = ctx.SimpleQueue()
    procs = []
    for r in range(nprocs):
        p = ctx.Process(target=_spawn_entry, args=(fn, r, tuple(args), err_q), daemon=False)
        p.start()
        procs.append(p)
    if not join:
        return procs
    try:
        while True:
            alive = [p for p in procs if p.is_alive()]
            failed = [(i, p) for i, p in enumerate(procs) if p.exitcode not in (None, 0)]
            if failed:
                for p in alive:
                    p.terminate()
                for p in procs:
                    p.join(10)
                rank, code = failed[0][0], failed[0][1].exitcode
                msg = f"process {rank} terminated with exit code {code}"
                if not err_q.empty():
                    r, tb = err_q.get()
                    msg = f"process {r} raised:\n{tb}"
                raise ProcessRaisedException(msg)
            if not alive:
                return None
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            p.terminate()
        raise


def _worker_env(base, *, rank, local_rank, world, local_world, node_rank, master_addr, master_port, restart,
                max_restarts, run_id):
    e = dict(base)
    e.update(RANK=str(rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(local_world),
             GROUP_RANK=str(node_rank), ROLE_RANK=str(rank), ROLE_WORLD_SIZE=str(world), ROLE_NAME="default",
             GROUP_WORLD_SIZE=str(world // local_world), MASTER_ADDR=master_addr, MASTER_PORT=str(master_port),
             TORCHELASTIC_RESTART_COUNT=str(restart), TORCHELASTIC_MAX_RESTARTS=str(max_restarts),
             TORCHELASTIC_RUN_ID=run_id)
    return e


def launch(cmd: list[str], nproc_per_node: int = 1, nnodes: int = 1, node_rank: int = 0,
           master_addr: str = "127.0.0.1", master_port: int = 29500, max_restarts: int = 0,
           monitor_interval: float = 0.1, run_id: str | None = None, timeout_s: float | None = None) -> int:
    """Run ``cmd`` (argv) as ``nproc_per_node`` workers; returns the group's exit code."""
    world = nproc_per_node * nnodes
    run_id = run_id or uuid.uuid4().hex[:8]
    base = dict(os.environ)
    if nproc_per_node > 1 and "OMP_NUM_THREADS" not in base:
        print("*****************************************\n"
              "Setting OMP_NUM_THREADS environment variable for each process to be 1 in default, to avoid your "
              "system being overloaded, please further tune the variable for optimal performance in your "
              "application as needed. \n*****************************************", file=sys.stderr)
        base["OMP_NUM_THREADS"] = "1"
    for restart in range(max_restarts + 1):
        procs = []
        for lr in range(nproc_per_node):
            r = node_rank * nproc_per_node + lr
            env = _worker_env(base, rank=r, local_rank=lr, world=world, local_world=nproc_per_node,
                              node_rank=node_rank, master_addr=master_addr, master_port=master_port,
                              restart=restart, max_restarts=max_restarts, run_id=run_id)
            procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
        t0 = time.time()
        code = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                code = bad[0]
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.time() - t0 > timeout_s:
                code = 124
                break
            time.sleep(monitor_interval)
        # a worker failed: tear the whole group down (no survivors stuck in a collective)
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        deadline = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
        print(f"[ptdt.launch] worker group failed (exit {code}); restart {restart}/{max_restarts}", file=sys.stderr)
    return code if code else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="torchrun-compatible single-node launcher")
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node-rank", "--node_rank", type=int, default=0)
    ap.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    ap.add_argument("--master-port", "--master_port", type=int, default=29500)
    ap.add_argument("--max-restarts", "--max_restarts", type=int, default=0)
    ap.add_argument("--run-id", "--run_id", default=None)
    ap.add_argument("--timeout", type=float, default=None, help="kill the group after this many seconds")
    ap.add_argument("-m", dest="module", default=None, help="run a module instead of a script")
    ap.add_argument("script", nargs="?")
    ap.add_argument("script_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.module:
        cmd = [sys.executable, "-m", a.module] + ([a.script] if a.script else []) + a.script_args
    else:
        cmd = [sys.executable, a.script] + a.script_args
    return launch(cmd, a.nproc_per_node, a.nnodes, a.node_rank, a.master_addr, a.master_port, a.max_restarts,
                  run_id=a.run_id, timeout_s=a.timeout)


if __name__ == "__main__":
    sys.exit(main())
