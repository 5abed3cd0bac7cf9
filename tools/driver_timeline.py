#!/usr/bin/env python3
"""Where the microseconds of the driver command go: a host + device timeline of the
bench's timed region (``bench.py --gpus 1 --steps 20 --warmup 5``, headline engine).

The bench's timed region is ``plan.launch_at(20, pos)`` (Python -> pybind -> C++ ->
hipLaunchKernel) followed by ``torch.cuda.synchronize()``. This probe builds the same
plan the bench builds and repeats that region ``--reps`` times, stamping

  host  (CLOCK_MONOTONIC): h0 before the Python call, the C++ launcher's stamps right
        before / after hipLaunchKernel (PersistentPlan.last_launch_ns), h1 when the call
        returned to Python, h2 when torch.cuda.synchronize() returned;
  device (100 MHz realtime counter, PersistArgs::tl, stored into host-mapped memory):
        kernel entry, past the prologue barrier, after the last step, after the final
        parameter / cursor stores.

Device stamps are moved onto the host axis by a ping calibration (native
``clock_calibrate``: the host flips a host-mapped flag, a 1-thread kernel answers with
its counter; the offset comes from the tightest round trips, +-rtt/2).

Variants (one JSON line each, medians over the reps, plus the calibration line):
  bench    the bench's exact sequence (comm.barrier + sync before, launch, torch sync)
  pinned   as bench, on a stream restricted to CU 0 (every launch lands where the previous one ran)
  spin     as bench, but the host first spins on the kernel's final stamp, then syncs
           (how long the synchronize takes once the kernel's last store is visible)
  hipsync  hipDeviceSynchronize straight from C++ instead of torch.cuda.synchronize
  nostamp  timeline off (the stamps' own cost: compare total_us with bench)
  idle2ms  as bench after a 2 ms host sleep (GPU idle before the launch)
  busyNNN  as bench after NNN us of host busy-waiting (GPU idle, CPU awake)
  cold     as bench after a 50 ms host sleep (GPU power state dropped)
  coldwN   as cold, then N ms of streaming kernels before the barrier (power-state ramp back up)
  benchexact  bench.py's own _timed() around the launch (window from its CLOCK_MONOTONIC stamps)
  waitK    launch + wait entirely in C++ (PersistentPlan.launch_wait_at mode K: 0 hipDeviceSynchronize,
           1 hipStreamSynchronize, 2 event record + synchronize, 3 hipExtLaunchKernel stop event +
           synchronize, 4 hipStreamQuery spin, 5 ext-launch stop event + hipEventQuery spin), then the
           bench's torch.cuda.synchronize()
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def calibrate(C, n=64):
    hs, hseen, dt = C.clock_calibrate(n)
    pings = [(b - a, (a + b) / 2 - 10 * t) for a, b, t in zip(hs, hseen, dt) if t > 0]
    if not pings:
        raise RuntimeError("clock calibration failed: the ping kernel never answered")
    pings.sort()
    best = pings[:max(4, len(pings) // 8)]
    off = statistics.median(o for _, o in best)
    return off, {"pings": len(pings), "rtt_min_us": round(pings[0][0] / 1e3, 3),
                 "rtt_med_us": round(statistics.median(r for r, _ in pings) / 1e3, 3),
                 "offset_spread_us": round((max(o for _, o in best) - min(o for _, o in best)) / 1e3, 3)}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--variants", default="bench,spin,hipsync,nostamp,idle2ms,busy20,busy100,busy500,"
                                          "wait0,wait1,wait2,wait3,wait4,wait5,cold,coldw0.2,coldw1,coldw5,benchexact")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)

    import bench
    from pytorch_distributed_training_tutorials_amd._ext import native
    from pytorch_distributed_training_tutorials_amd.data.device_sampler import DeviceDistributedSampler
    from pytorch_distributed_training_tutorials_amd.ops.fused_step import FusedMLPStep
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod

    C = native()
    args = bench.parse(["--steps", str(a.steps), "--warmup", str(a.warmup)])
    rank, world, local = bench._setup(args, False)
    dev = torch.device("cuda", local)
    comm = comm_mod.get_default(dev)
    model, loss = bench._build_model(args, dev)
    ds = bench._dataset(args, dev, loss)
    X, Y = ds.tensors
    eng = FusedMLPStep(model, loss=loss, lr=args.lr, comm=comm)
    sampler = DeviceDistributedSampler(len(ds), world, rank, seed=args.seed, device=dev)
    cursor = torch.zeros(2, dtype=torch.int32, device=dev)
    losses = torch.zeros(max(a.steps, a.warmup, 1), device=dev)
    plan = eng.persistent_plan(X, Y, args.batch_size, sampler, cursor, losses)
    hm = C.HostMapped(8)
    # "pinned": the bench sequence on a stream restricted to CU 0 (hipExtStreamCreateWithCUMask), so every
    # launch finds the previous one's instruction cache, L1 / TLB and XCD L2 state
    pin = torch.cuda.ExternalStream(C.cu_masked_stream(dev.index, [0]), device=dev) if "pinned" in a.variants else None
    warm = torch.empty(64 << 20, device=dev)  # 256 MiB for the power-state ramp variants
    pos = 0
    plan.launch_at(a.warmup, pos)
    pos += a.warmup
    torch.cuda.synchronize(dev)

    off, cal = calibrate(C)
    lines = [{"what": "calibration", **cal}]

    def dev_ns(t):
        return 10 * t + off

    for var in a.variants.split(","):
        rows, first = [], []
        for r in range(a.reps + 2):
            hm.zero()
            plan.set_timeline(0 if var == "nostamp" else hm.device_ptr)
            if var.startswith("cold"):
                time.sleep(0.05)
                if var.startswith("coldw"):  # ~N ms of HBM streaming (2 x 256 MiB per add_, ~0.1 ms each)
                    for _ in range(max(1, int(float(var[5:]) * 10))):
                        warm.add_(1.0)
            if var == "benchexact":
                torch.cuda.synchronize(dev)
                bench._timed(comm, dev, lambda: plan.launch_at(a.steps, pos), label="tl")
                h2 = None
            comm.barrier()
            torch.cuda.synchronize(dev)
            if var == "idle2ms":
                time.sleep(0.002)
            elif var.startswith("busy"):
                t_end = C.mono_ns() + 1000 * int(var[4:])
                while C.mono_ns() < t_end:
                    pass
            seen = None
            waited = None
            if var == "benchexact":  # the launch already ran inside bench._timed
                w_us = bench._TIMINGS["tl"]["window_us"]
                pos += a.steps
                if r >= 2:
                    rows.append({"total_us": w_us})
                else:
                    first.append({"total_us": w_us})
                continue
            if var.startswith("wait"):
                h0, h1, waited = plan.launch_wait_at(a.steps, pos, int(var[4:]))
                torch.cuda.synchronize(dev)
                h2 = C.mono_ns()
            elif var == "pinned":
                with torch.cuda.stream(pin):
                    h0 = C.mono_ns()
                    plan.launch_at(a.steps, pos)
                    h1 = C.mono_ns()
                    torch.cuda.synchronize(dev)
                    h2 = C.mono_ns()
            else:
                h0 = C.mono_ns()
                plan.launch_at(a.steps, pos)
                h1 = C.mono_ns()
                if var == "spin":
                    seen = hm.spin(3, 1_000_000_000)
                if var == "hipsync":
                    h2 = C.hip_device_sync_ns()
                else:
                    torch.cuda.synchronize(dev)
                    h2 = C.mono_ns()
            pos += a.steps
            l0, l1 = plan.last_launch_ns()
            if var in ("wait3", "wait5"):  # hipExtLaunchKernel: no launcher stamps
                l0, l1 = h0, h1
            tl = hm.read()
            row = {"total_us": (h2 - h0) / 1e3, "py_to_hip_call_us": (l0 - h0) / 1e3,
                   "hipLaunchKernel_us": (l1 - l0) / 1e3, "hip_return_to_py_us": (h1 - l1) / 1e3}
            if var != "nostamp" and all(t > 0 for t in tl[:4]):
                e, b, s_end, x = (dev_ns(t) for t in tl[:4])
                row.update({
                    "launch_call_to_kernel_entry_us": (e - l0) / 1e3,
                    "prologue_entry_to_barrier_us": (b - e) / 1e3,
                    "steps_barrier_to_last_us": (s_end - b) / 1e3,
                    "epilogue_stores_us": (x - s_end) / 1e3,
                    "kernel_end_to_sync_return_us": (h2 - x) / 1e3,
                    "kernel_entry_to_end_us": (x - e) / 1e3,
                })
                if waited is not None:
                    row["wait_returned_after_end_us"] = (waited - x) / 1e3
                    row["torch_sync_after_wait_us"] = (h2 - waited) / 1e3
                if seen is not None and seen > 0:
                    row["end_store_seen_by_host_us"] = (seen - x) / 1e3
                    row["sync_after_seen_us"] = (h2 - seen) / 1e3
            if r < 2:  # first reps of a variant: reported apart (full breakdown), not in the medians
                first.append({k: round(v, 3) for k, v in row.items()})
                continue
            rows.append(row)
        keys = rows[0].keys()
        med = {k: round(statistics.median(rw[k] for rw in rows if k in rw), 3) for k in keys}
        lo = {k: round(min(rw[k] for rw in rows if k in rw), 3) for k in ("total_us",)}
        lines.append({"what": "timeline", "variant": var, "steps": a.steps, "reps": len(rows), "median": med,
                      "min_total_us": lo["total_us"], "first_reps": first})
    for ln in lines:
        s = json.dumps(ln)
        print(s, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(s + "\n")
    plan.set_timeline(0)
    from pytorch_distributed_training_tutorials_amd.parallel.env import destroy_process_group

    destroy_process_group()


if __name__ == "__main__":
    main()
