"""How torch.autocast(bfloat16) evaluates F.cross_entropy on bf16 logits (probe)."""
import torch
import torch.nn.functional as F

dev = torch.device("cuda", 0)
torch.manual_seed(0)
z = (torch.randn(32, 10, device=dev) * 2).to(torch.bfloat16).requires_grad_(True)
y = torch.randint(0, 10, (32,), device=dev)
with torch.autocast("cuda", dtype=torch.bfloat16):
    l_ac = F.cross_entropy(z, y)
    ls_ac = torch.log_softmax(z, 1)
    print("autocast: loss dtype", l_ac.dtype, "log_softmax dtype", ls_ac.dtype)
(g_ac,) = torch.autograd.grad(l_ac, z)
l_32 = F.cross_entropy(z.float(), y)
l_bf = F.cross_entropy(z, y)  # no autocast: bf16 math
print("loss autocast", float(l_ac), "fp32", float(l_32), "bf16-noautocast", float(l_bf))
zf = z.detach().float().requires_grad_(True)
(g_32,) = torch.autograd.grad(F.cross_entropy(zf, y), zf)
(g_bfna,) = torch.autograd.grad(F.cross_entropy(z, y), z)
print("grad dtype", g_ac.dtype, "max|g_ac - bf16(g_fp32)|", (g_ac.float() - g_32.to(torch.bfloat16).float()).abs().max().item(),
      "max|g_ac - g_bf16math|", (g_ac.float() - g_bfna.float()).abs().max().item())
