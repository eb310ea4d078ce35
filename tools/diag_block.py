"""Single ConvBlock(+BN+ReLU) gradients vs float64 (isolates the layer kernels)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from dgvcc_amd.models.models import ConvBlock
dev = torch.device("cuda")
torch.manual_seed(0)
for (N, C, Co, H, W, relu) in [(2, 256, 128, 16, 16, True), (2, 512, 256, 16, 16, True), (2, 256, 128, 16, 16, False), (2, 64, 64, 32, 32, True)]:
    blk = ConvBlock(C, Co, bn=True, relu=relu)
    with torch.no_grad():
        blk.bn.weight.uniform_(0.5, 1.5); blk.bn.bias.uniform_(-0.2, 0.2)
    x = torch.relu(torch.randn(N, C, H, W))
    g = torch.randn(N, Co, H, W)
    def ref(dtype):
        xx = x.to(dtype).requires_grad_(True)
        w = blk.conv.weight.detach().to(dtype).requires_grad_(True)
        ga = blk.bn.weight.detach().to(dtype).requires_grad_(True)
        be = blk.bn.bias.detach().to(dtype).requires_grad_(True)
        y = F.conv2d(xx, w, padding=1)
        y = F.batch_norm(y, None, None, ga, be, True, 0.1, 1e-5)
        if relu: y = F.relu(y)
        y.backward(g.to(dtype))
        return y.detach(), xx.grad, w.grad, ga.grad, be.grad
    r64 = ref(torch.float64); r32 = ref(torch.float32)
    b = blk.to(dev).train()
    xd = x.to(dev).detach().requires_grad_(True)
    y = b(xd)
    print("leaf", xd.is_leaf, "y.grad_fn", y.grad_fn, flush=True)
    y.backward(g.to(dev))
    print("xd.grad", None if xd.grad is None else xd.grad.shape, "w.grad", None if b.conv.weight.grad is None else b.conv.weight.grad.shape, flush=True)
    mine = (y.detach().cpu(), xd.grad.cpu(), b.conv.weight.grad.cpu(), b.bn.weight.grad.cpu(), b.bn.bias.grad.cpu())
    def e(a, r): return ((a.double() - r.double()).norm() / r.double().norm()).item()
    print(f"N{N} C{C}->{Co} {H}x{W} relu={relu}")
    for name, a, c32, c64 in zip(["y", "dx", "dw", "dgamma", "dbeta"], mine, r32, r64):
        print(f"   {name:7s} hip {e(a, c64):.2e}  cpu32 {e(c32, c64):.2e}")
    blk.cpu()
