import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from dgvcc_amd.models.models import ConvBlock
from dgvcc_amd import engine as E, kernels as K
dev = torch.device("cuda")
torch.manual_seed(0)
N, C, Co, H, W = 2, 512, 256, 16, 16
blk = ConvBlock(C, Co, bn=True, relu=True)
with torch.no_grad():
    blk.bn.weight.uniform_(0.5, 1.5); blk.bn.bias.uniform_(-0.2, 0.2)
blk = blk.to(dev)
x = torch.relu(torch.randn(N, C, H, W, device=dev))
g = torch.randn(N, Co, H, W, device=dev)
layer = E.ConvLayer(blk.conv, blk.bn, E.ACT_RELU)
tape = {}
xa = K.Act(x.permute(0, 2, 3, 1).contiguous())
out = K.Act(K.nhwc(N, H, W, Co, torch.float32, dev))
layer.forward(xa, out, True, tape)
xx, z, stats, wp, drop, tr = tape[layer]
zref = F.conv2d(x, blk.conv.weight, padding=1)
print("z err", ((z.buf.permute(0,3,1,2) - zref).norm() / zref.norm()).item())
mu = zref.mean((0,2,3)); var = zref.var((0,2,3), unbiased=False)
print("mean err", ((stats[0]-mu).norm()/mu.norm()).item(), "invstd err", ((stats[1]-torch.rsqrt(var+1e-5)).norm()/stats[1].norm()).item())
zr = zref.detach().clone().requires_grad_(True)
yr = F.relu(F.batch_norm(zr, None, None, blk.bn.weight, blk.bn.bias, True, 0.1, 1e-5))
print("y err", ((out.buf.permute(0,3,1,2) - yr).norm()/yr.norm()).item())
yr.backward(g)
ga = K.Act(g.permute(0, 2, 3, 1).contiguous())
dz = K.Act(torch.empty_like(z.buf)); dgam = torch.empty(Co, device=dev); dbet = torch.empty(Co, device=dev)
K.bn_bwd(ga, z, blk.bn.weight.detach(), stats, 1, dz, dgam, dbet)
torch.cuda.synchronize()
print("dz err", ((dz.buf.permute(0,3,1,2) - zr.grad).norm()/zr.grad.norm()).item())
gb = blk.bn.bias.grad if blk.bn.bias.grad is not None else None
ref_dbet = (g * (yr > 0)).sum((0,2,3))
print("dbeta err", ((dbet - ref_dbet).norm()/ref_dbet.norm()).item())
grads = layer.backward(tape, ga, K.Act(torch.empty_like(xx.buf)))
print("layer dbeta err", ((grads[blk.bn.bias] - ref_dbet).norm()/ref_dbet.norm()).item())
