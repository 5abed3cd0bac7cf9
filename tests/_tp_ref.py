"""Plain-PyTorch references for the bf16 tensor-parallel engine (csrc/kernels/mlp_tp_impl.h, BF):
the toy MLP's DDP steps with explicit bf16 rounding at torch.autocast(bfloat16)'s rounding points
("emulate"), or in plain fp32 ("fp32"); W ranks' per-rank gradients averaged in rank order like
the DDP all-reduce. Reference training step: ddp_gpus_torchrun.py:30-35."""
import torch


def bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).float()


def _loss_grad(z, y, loss, nb, dout, emulate=False):
    """(loss, dL/dz) in fp32 for logits z [nb, dout]. ``emulate``: cross-entropy the way
    torch.autocast(bfloat16) evaluates it on bf16 logits -- a bf16 log_softmax, the nll / soft-target
    sum in fp32 on those values, and a bf16 log_softmax backward dz = bf16(g - exp(ls) sum(g)) with
    g = bf16(dL/dls) (scripts/r6/ce_probe.py: autocast's gradient equals that bf16 math exactly)."""
    if emulate and loss != "mse":
        ls = bf(torch.log_softmax(z, 1))
        if loss == "ce_soft":
            l = -(ls * y).sum() / nb
            g = bf(-y / nb)
        else:
            keep = y != -100
            cnt = int(keep.sum())
            yy = torch.where(keep, y, torch.zeros_like(y))
            oh = torch.nn.functional.one_hot(yy, dout).float() * keep[:, None].float()
            l = -(ls * oh).sum() / max(cnt, 1)
            g = bf(-oh * (1.0 / max(cnt, 1)))
        return l, bf(g - torch.exp(ls) * g.sum(1, keepdim=True))
    if loss == "mse":
        d = z - y
        return (d * d).sum() / (nb * dout), 2.0 * d / (nb * dout)
    if loss == "ce_soft":
        ls = torch.log_softmax(z, 1)
        return -(y * ls).sum() / nb, (torch.softmax(z, 1) * y.sum(1, keepdim=True) - y) / nb
    keep = y != -100
    cnt = int(keep.sum())
    yy = torch.where(keep, y, torch.zeros_like(y))
    ls = torch.log_softmax(z, 1)
    oh = torch.nn.functional.one_hot(yy, dout).float()
    g = (torch.softmax(z, 1) - oh) * keep[:, None].float() / max(cnt, 1)
    return -(ls.gather(1, yy[:, None])[:, 0] * keep.float()).sum() / max(cnt, 1), g


def ddp_reference(params, X, Y, orders, B, loss, steps, lr, mom, mode="emulate"):
    """params: [W1, b1, W2, b2] (b's may be None); orders[r][e]: rank r's index list of epoch e.
    Returns (params, last averaged grads, per-step losses of rank 0)."""
    W1, b1, W2, b2 = [None if p is None else p.detach().clone().float() for p in params]
    ps = [p for p in (W1, b1, W2, b2) if p is not None]
    bufs = [None] * len(ps)
    world = len(orders)
    ns = orders[0][0].numel()
    S = -(-ns // B)
    r = bf if mode == "emulate" else (lambda t: t)
    dout = W2.shape[0]
    losses, grads = [], None
    for k in range(steps):
        e, j = divmod(k, S)
        acc = None
        for rank in range(world):
            idx = orders[rank][e][j * B:(j + 1) * B].long()
            x, y = r(X[idx]), Y[idx]
            nb = idx.numel()
            pre = x @ r(W1).T + (r(b1) if b1 is not None else 0)
            h = r(torch.relu(pre))
            z = r(h @ r(W2).T + (r(b2) if b2 is not None else 0))
            l, dz = _loss_grad(z, y, loss, nb, dout, mode == "emulate")
            dz = r(dz)
            g = [None, None, r(dz.T @ h), r(dz.sum(0)) if b2 is not None else None]
            dh = r(dz @ r(W2)) * (h > 0).float()
            g[0] = r(dh.T @ x)
            g[1] = r(dh.sum(0)) if b1 is not None else None
            g = [t for t in g if t is not None]
            acc = g if acc is None else [a + t for a, t in zip(acc, g)]
            if rank == 0:
                losses.append(float(l))
        grads = [a / world for a in acc]
        for i, (p, gr) in enumerate(zip(ps, grads)):
            if mom:
                bufs[i] = gr.clone() if bufs[i] is None else mom * bufs[i] + gr
                gr = bufs[i]
            p -= lr * gr
    return ps, grads, losses
