"""Whole-step hipGraph capture (utils/graphs.py): a DDP ResNet-50 training step
(native conv weight casts with grad sinks, fused BN, DDP reducer, FusedSGD with
bf16 shadows) replayed from one captured graph follows the same trajectory as the
same steps launched eagerly."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    from pytorch_distributed_training_tutorials_amd.parallel import env

    env.init_process_group("nccl")
    yield
    env.destroy_process_group()


def _run(dev, graphed: bool, steps: int, init_state):
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    comm = comm_mod.get_default(dev)
    model = resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    model.load_state_dict(init_state)
    ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
    opt = FusedSGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(4, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), generator=g).to(dev)

    def step():
        ddp.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=not graphed):
            out = ddp(x)
        loss = cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    losses = []
    if graphed:
        warm = 2
        # the warm-up steps are training steps; record their losses through a wrapper
        def rec():
            loss = step()
            losses.append(loss.detach().clone())
            return loss

        gs = GraphedStep(rec, dev, comm=comm, warmup=warm)
        losses.pop()  # the capture call's (never executed) loss tensor
        for _ in range(steps - warm):
            losses.append(gs().detach().clone())
        assert gs.n_collectives == 0  # world 1: the reducer issues no collective
    else:
        for _ in range(steps):
            losses.append(step().detach().clone())
    torch.cuda.synchronize(dev)
    return [float(v) for v in losses], {k: v.detach().float().cpu() for k, v in model.state_dict().items()}


def test_col_sum_replay_after_eager_launches(dev, native):
    """The Linear bias-gradient column sum replayed from a graph after eager launches of the same op
    (the round-3 ResNet divergence: the captured zero-fill of its accumulator stopped being applied
    once eager steps had run between replays, so fc.bias's gradient summed onto stale memory)."""
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(128, 1000, generator=g).to(dev, torch.bfloat16)
    out = torch.empty(1000, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        native.col_sum_(x, out, False)
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize(dev)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        native.col_sum_(x, out, False)
    torch.cuda.synchronize(dev)
    want = x.float().sum(0)
    for rnd in range(3):
        for _ in range(4):  # eager launches of the op on other buffers
            x2 = torch.randn(128, 1000, device=dev, dtype=torch.bfloat16)
            o2 = torch.full((1000,), 123.0, device=dev)
            native.col_sum_(x2, o2, False)
            torch.testing.assert_close(o2, x2.float().sum(0), rtol=1e-4, atol=1e-3)
        out.fill_(7e30)
        graph.replay()
        torch.cuda.synchronize(dev)
        torch.testing.assert_close(out, want, rtol=1e-4, atol=1e-3, msg=lambda m: f"round {rnd}: {m}")


def test_graph_memset_nodes_replaced(dev, native):
    """GraphedStep rewrites a captured hipMemsetAsync into a fill-kernel node before instantiation
    (csrc/kernels/graph_memset.hip; profiles/r4_graph_memset.md) and the replay still zeroes the buffer,
    also after eager memsets of other buffers."""
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    buf = torch.full((1000,), 7.0, device=dev)
    half = torch.full((4099,), 3, dtype=torch.int16, device=dev)  # odd byte count

    def fn():
        native.memset_async_(buf, 0)
        buf.add_(1.0)
        native.memset_async_(half, 0)
        half.add_(2)

    gs = GraphedStep(fn, dev, warmup=1)
    assert gs.memset_nodes >= 2 and gs.memsets_replaced == gs.memset_nodes
    other = torch.empty(4096, device=dev)
    for _ in range(3):
        native.memset_async_(other, 0)  # eager memsets between replays
        buf.fill_(5.0)
        half.fill_(9)
        gs()
        torch.cuda.synchronize(dev)
        assert bool((buf == 1.0).all()) and bool((half == 2).all())


def test_col_sum_deterministic(dev, native):
    """Bias gradients are fixed-order sums: bit-identical across launches (no atomics)."""
    for rows, cols in ((128, 1000), (32, 1), (20000, 96), (3, 4100)):
        x = torch.randn(rows, cols, device=dev, dtype=torch.bfloat16)
        a = torch.empty(cols, device=dev)
        b = torch.empty(cols, device=dev)
        native.col_sum_(x, a, False)
        native.col_sum_(x, b, False)
        assert torch.equal(a, b)
        torch.testing.assert_close(a, x.double().sum(0).float(), rtol=1e-4, atol=2e-3)
        c = torch.ones(cols, device=dev)
        native.col_sum_(x, c, True)
        torch.testing.assert_close(c, a + 1, rtol=1e-5, atol=1e-4)


def _interleaved(dev, pattern: str, init_state, lr: float = 0.05, warm: int = 2):
    """One trajectory: ``warm`` eager warm-up steps inside GraphedStep, then ``pattern`` (E = eager
    step, R = graph replay) -- benchmarks/resnet_ddp.py's --graph auto A/B does exactly this."""
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.utils.graphs import GraphedStep

    comm = comm_mod.get_default(dev)
    model = resnet50(num_classes=10).to(dev).to(memory_format=torch.channels_last)
    model.load_state_dict(init_state)
    ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
    opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(4, 3, 64, 64, generator=g).to(dev).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (4,), generator=g).to(dev)
    losses = []

    def step():
        ddp.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
            out = ddp(x)
        loss = cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        if not torch.cuda.is_current_stream_capturing():  # a capture executes nothing
            losses.append(loss.detach().clone())
        return loss

    if "R" in pattern:
        gs = GraphedStep(step, dev, comm=comm, warmup=warm)
    else:
        gs = None
        pattern = "E" * warm + pattern
    for c in pattern:
        if c == "E":
            step() if gs is None else gs.eager()
        else:
            losses.append(gs().detach().clone())
    torch.cuda.synchronize(dev)
    return [float(v) for v in losses], {k: v.detach().float().cpu() for k, v in model.state_dict().items()}


def test_interleaved_eager_and_replay_matches_pure_eager(pg, dev):
    """E E R R E E R R ... (18 steps after warm-up; eager steps through GraphedStep.eager, which
    re-captures before the next replay) follows the pure-eager trajectory."""
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    torch.manual_seed(0)
    init = {k: v.clone() for k, v in resnet50(num_classes=10).state_dict().items()}
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        pat = "EERR" * 4 + "ER"
        la, sa = _interleaved(dev, "E" * len(pat), init)
        lb, sb = _interleaved(dev, pat, init)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    assert len(la) == len(lb) == len(pat) + 2
    assert all(torch.isfinite(torch.tensor(lb)))
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=2e-3, atol=2e-3)
    for k in sa:
        torch.testing.assert_close(sb[k], sa[k], rtol=2e-3, atol=2e-3, msg=lambda m, k=k: f"{k}: {m}")


def test_graphed_resnet_ddp_step_matches_eager(pg, dev):
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50

    torch.manual_seed(0)
    init = {k: v.clone() for k, v in resnet50(num_classes=10).state_dict().items()}
    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        la, sa = _run(dev, False, 6, init)
        lb, sb = _run(dev, True, 6, init)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    assert len(la) == len(lb) == 6
    assert all(torch.isfinite(torch.tensor(la)))
    # replays must keep training: the loss moves, and equals the eager trajectory
    assert la[-1] != la[0]
    torch.testing.assert_close(torch.tensor(lb), torch.tensor(la), rtol=2e-3, atol=2e-3)
    for k in sa:
        torch.testing.assert_close(sb[k], sa[k], rtol=2e-3, atol=2e-4, msg=lambda m, k=k: f"{k}: {m}")


def test_graph_replay_with_miopen_memset_nodes_tracks_eager(pg, dev):
    """The configuration that diverged: exhaustive-find MIOpen solvers
    (cudnn.benchmark=True) whose atomic weight-gradient kernels zero their outputs with
    hipMemsetAsync, so the captured ResNet-50 step holds memset nodes. GraphedStep rewrites every one
    (memsets_replaced == memset_nodes > 0) and 4 replays from a snapshot follow 4 eager steps from the
    same snapshot within 2e-3 (benchmarks/graph_memset_probe.py: without the rewrite the 2nd replay's
    loss is ~1e19; profiles/r5_graph_memset.md)."""
    from pytorch_distributed_training_tutorials_amd import native
    from pytorch_distributed_training_tutorials_amd.models.resnet import resnet50
    from pytorch_distributed_training_tutorials_amd.ops.loss import cross_entropy
    from pytorch_distributed_training_tutorials_amd.ops.optim import FusedSGD
    from pytorch_distributed_training_tutorials_amd.parallel import comm as comm_mod
    from pytorch_distributed_training_tutorials_amd.parallel.ddp import DistributedDataParallel
    from pytorch_distributed_training_tutorials_amd.utils import graphs

    old = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = False, True
    try:
        comm = comm_mod.get_default(dev)
        torch.manual_seed(0)
        model = resnet50(num_classes=1000).to(dev).to(memory_format=torch.channels_last)
        ddp = DistributedDataParallel(model, device_ids=[dev.index], comm=comm)
        # small steps: the atomic solvers' run-to-run noise stays far below the tolerance (at lr 0.1
        # two EAGER runs from one snapshot already differ by ~5 % after 4 steps)
        opt = FusedSGD(model.parameters(), lr=0.002, momentum=0.9, weight_decay=1e-4, bf16_shadow=True)
        x = torch.empty(32, 3, 128, 128, device=dev)
        native().philox_(x, 1234, 0, 1)
        x = x.contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(5))

        def step():
            ddp.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
                out = ddp(x)
            loss = cross_entropy(out.float(), y)
            loss.backward()
            opt.step()
            return loss

        gs = graphs.GraphedStep(step, dev, comm=comm, warmup=3)
        assert gs.memset_nodes > 0, "no memset node captured: the test no longer covers the failing path"
        assert gs.memsets_replaced == gs.memset_nodes
        live = [p.data for p in model.parameters()]
        live += [sh for p in model.parameters() if (sh := getattr(p, "_ptdt_bf16", None)) is not None]
        live += [opt.state[p]["momentum_buffer"] for p in model.parameters() if "momentum_buffer" in opt.state.get(p, {})]
        live += list(model.buffers()) + list(opt._counters.values()) + list(ddp.reducer.bucket_tensors())
        snap = [t.detach().clone() for t in live]
        rl = [float(gs()) for _ in range(4)]
        torch.cuda.synchronize(dev)
        with torch.no_grad():
            for t, s in zip(live, snap):
                t.copy_(s)
        el = [float(step()) for _ in range(4)]
        torch.cuda.synchronize(dev)
        with torch.no_grad():
            for t, s in zip(live, snap):
                t.copy_(s)
        el2 = [float(step()) for _ in range(4)]  # eager again: the atomic solvers' run-to-run floor
        torch.cuda.synchronize(dev)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = old
    rl, el, el2 = torch.tensor(rl), torch.tensor(el), torch.tensor(el2)
    assert bool(torch.isfinite(rl).all())
    gap = ((rl - el).abs() / el.abs()).max().item()
    floor = ((el2 - el).abs() / el.abs()).max().item()
    print(f"replay vs eager {gap:.2e}, eager vs eager {floor:.2e}, memset nodes {gs.memset_nodes}")
    # the first replay's forward runs the snapshot's weights: same loss as the eager step's
    assert abs(rl[0] - el[0]) <= 1e-3 * abs(el[0])
    # then within 2e-3, or within the noise two eager runs show (the atomic solvers' order differs
    # run to run; measured 3-9e-3 after 4 steps); without the rewrite the loss is ~1e19 by replay 2
    assert gap <= max(2e-3, 5 * floor) and gap < 0.05, (gap, floor)


# the memset nodes of the captured ResNet-50 step (benchmarks/graph_memset_probe.py): value 0, byte
# elements, (width, dst offset mod 4 KiB)
_RESNET_MEMSETS = [(131072, 3584)] * 4 + [(131072, 0)] * 3 + [(65536, 0), (32768, 3584), (32768, 3584), (8192, 3584)]


def test_graph_memset_nodes_fail_from_the_second_replay_and_the_rewrite_fixes_it(dev, native):
    """Root cause of the replay divergence (profiles/r5_graph_memset.md): a graph holding the captured
    step's memset shapes -- hipMemsetAsync calls only, no MIOpen, no eager work in between -- zeroes
    every buffer on its first launch, but from the second launch on the runtime leaves thousands of
    bytes of several memset nodes unset. The same graph with the nodes rewritten as fill kernels
    (graph_replace_memsets, what GraphedStep does) is correct on every launch."""
    views, bufs = [], []
    for width, align in _RESNET_MEMSETS:
        b = torch.empty(width + 8192, dtype=torch.uint8, device=dev)
        off = (align - b.data_ptr()) % 4096
        bufs.append(b)
        views.append(b[off:off + width])
    other = torch.empty(3 * 4096 + 100, dtype=torch.uint8, device=dev)

    def run(rewrite: bool):
        side = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g, stream=side):
            for v in views:
                native.memset_async_(v, 0)
            native.memset_async_(other, 0x3F)
        raw = g.raw_cuda_graph()
        if rewrite:
            assert native.graph_replace_memsets(raw) == len(views) + 1
        g.instantiate()
        bad = []
        for _ in range(4):
            for v in views:
                v.fill_(0xAB)
            other.fill_(0)
            torch.cuda.synchronize(dev)
            g.replay()
            torch.cuda.synchronize(dev)
            bad.append(sum(int((v != 0).sum()) for v in views) + int((other != 0x3F).sum()))
        return bad

    fixed = run(True)
    assert fixed == [0, 0, 0, 0]
    raw = run(False)  # the runtime's own memset nodes: reported, not asserted (a fixed runtime passes too)
    print("unset bytes per launch, memset nodes kept:", raw, "rewritten:", fixed)
