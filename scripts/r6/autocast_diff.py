"""One toy-MLP step: torch.autocast(bfloat16) gradients vs the bf16 emulation (tests/_tp_ref.py)."""
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, ".")
from tests._tp_ref import bf, _loss_grad  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(3)
B, Din, H, Dout = 32, 20, 64, 10
m = nn.Sequential(nn.Linear(Din, H), nn.ReLU(), nn.Linear(H, Dout)).to(dev)
X = torch.randn(B, Din, device=dev)
Y = torch.randint(0, Dout, (B,), device=dev)
acts = {}
m[0].register_forward_hook(lambda mod, i, o: acts.__setitem__("pre", o))
m[1].register_forward_hook(lambda mod, i, o: acts.__setitem__("h", o))
with torch.autocast("cuda", dtype=torch.bfloat16):
    z = m(X)
    l = F.cross_entropy(z, Y)
for t in ("pre", "h"):
    acts[t].retain_grad()
z.retain_grad()
l.backward()
W1, b1, W2, b2 = [p.detach() for p in m.parameters()]
x = bf(X)
pre = x @ bf(W1).T + bf(b1)
h = bf(torch.relu(pre))
ze = bf(h @ bf(W2).T + bf(b2))
le, dz = _loss_grad(ze, Y, "ce_index", B, Dout)
dz = bf(dz)
gW2, gb2 = bf(dz.T @ h), bf(dz.sum(0))
dh = bf(dz @ bf(W2)) * (h > 0).float()
gW1, gb1 = bf(dh.T @ x), bf(dh.sum(0))
print("dtypes", z.dtype, acts["pre"].dtype, acts["h"].dtype, "grad dtypes", z.grad.dtype, acts["h"].grad.dtype)
print("pre", (acts["pre"].float() - bf(pre)).abs().max().item(), "h", (acts["h"].float() - h).abs().max().item())
print("z", (z.float() - ze).abs().max().item(), "loss", float(l), float(le))
print("dz", (z.grad.float() - dz).abs().max().item(), "dh", (acts["h"].grad.float() - bf(dz @ bf(W2))).abs().max().item())
for n, a, b in (("W1", m[0].weight.grad, gW1), ("b1", m[0].bias.grad, gb1), ("W2", m[2].weight.grad, gW2),
                ("b2", m[2].bias.grad, gb2)):
    print(n, a.dtype, "maxdiff", (a - b).abs().max().item(), "max", b.abs().max().item())
# fp32 unrounded grads for scale
print("gW1 fp32-unrounded diff", (m[0].weight.grad - (dh.T @ x)).abs().max().item())
