import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from dgvcc_amd.models.models import ConvBlock
from dgvcc_amd import engine as E, kernels as K
dev = torch.device("cuda")
torch.manual_seed(0)
res = []
for (N, C, Co, H, W) in [(2, 256, 128, 16, 16), (2, 512, 256, 16, 16)]:
    blk = ConvBlock(C, Co, bn=True, relu=True)
    with torch.no_grad():
        blk.bn.weight.uniform_(0.5, 1.5); blk.bn.bias.uniform_(-0.2, 0.2)
    x = torch.relu(torch.randn(N, C, H, W))
    g = torch.randn(N, Co, H, W)
    res.append((blk, x, g))
blk, x, g = res[1]
N, C, H, W = x.shape
Co = g.shape[1]
# float64 reference
xx = x.double().requires_grad_(True)
w64 = blk.conv.weight.detach().double().requires_grad_(True)
ga = blk.bn.weight.detach().double().requires_grad_(True); be = blk.bn.bias.detach().double().requires_grad_(True)
y64 = F.relu(F.batch_norm(F.conv2d(xx, w64, padding=1), None, None, ga, be, True, 0.1, 1e-5))
y64.backward(g.double())
blk = blk.to(dev)
# direct layer path
layer = E.ConvLayer(blk.conv, blk.bn, E.ACT_RELU)
tape = {}
xa = K.Act(x.to(dev).permute(0, 2, 3, 1).contiguous())
out = K.Act(K.nhwc(N, H, W, Co, torch.float32, dev))
layer.forward(xa, out, True, tape)
gr = layer.backward(tape, K.Act(g.to(dev).permute(0, 2, 3, 1).contiguous()), K.Act(torch.empty_like(xa.buf)))
e = lambda a, r: ((a.double().cpu() - r.double()).norm() / r.double().norm()).item()
print("direct: y", e(out.buf.permute(0,3,1,2), y64), "dbeta", e(gr[blk.bn.bias], be.grad), "dgamma", e(gr[blk.bn.weight], ga.grad))
# autograd path
xd = x.to(dev).requires_grad_(True)
y = blk(xd)
y.backward(g.to(dev))
print("autograd: y", e(y, y64), "dbeta", e(blk.bn.bias.grad, be.grad), "dgamma", e(blk.bn.weight.grad, ga.grad), "dx", e(xd.grad, xx.grad))
# count relu-boundary elements
z64 = F.batch_norm(F.conv2d(x.double(), blk.conv.weight.detach().double().cpu(), padding=1), None, None, blk.bn.weight.detach().double().cpu(), blk.bn.bias.detach().double().cpu(), True, 0.1, 1e-5)
print("min |pre-relu|", z64.abs().min().item(), "count<1e-5", (z64.abs() < 1e-5).sum().item())
