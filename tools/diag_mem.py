import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from dgvcc_amd import engine as E, kernels as K
dev = torch.device("cuda")
g = torch.Generator().manual_seed(0)
N, k, S, h, w = 2, 256, 1024, 16, 16
mem = torch.nn.Parameter(torch.randn(1, k, S, generator=g).to(dev))
y = torch.relu(torch.randn(N, h, w, k, generator=g)).to(dev)
gyn = torch.randn(N, h, w, k, generator=g).to(dev)
mr = E.MemRead(mem)
dt = torch.float32
memT_s, mem_p, scale = mr.packs(dt)
ya = K.Act(y.contiguous())
L = mr.logits(ya, memT_s, dt)
P = K.Act(torch.empty_like(L.buf))
K.call("dg_softmax_fwd", L.dt, L.ptr, L.M, L.C, P.ptr, K.stream())
yn = mr.readout(P, mem_p, dt)
# torch reference in float64
m64 = mem.detach().double().requires_grad_(True)
y64 = y.double().permute(0, 3, 1, 2).contiguous().requires_grad_(True)
mk = m64.repeat(N, 1, 1).transpose(1, 2)
lg = torch.bmm(mk, y64.view(N, k, -1)) / 16
Pr = F.softmax(lg, 1)
ynr = torch.bmm(mk.transpose(1, 2), Pr).view(N, k, h, w)
e = lambda a, r: ((a.double() - r.double()).norm() / r.double().norm()).item()
print("logits", e(L.buf.view(N, h * w, S).transpose(1, 2), lg))
print("P", e(P.buf.view(N, h * w, S).transpose(1, 2), Pr))
print("ynew", e(yn.buf.permute(0, 3, 1, 2), ynr))
ynr.backward(gyn.double().permute(0, 3, 1, 2))
gP, da = mr.bwd_readout(K.Act(gyn.contiguous()), P, dt)
gL = K.Act(torch.empty_like(gP.buf))
K.call("dg_softmax_bwd", gP.dt, P.ptr, gP.ptr, gP.M, gP.C, gL.ptr, K.stream())
gy, db = mr.bwd_logits(gL, ya, mem_p, scale, dt)
print("dy", e(gy.buf.permute(0, 3, 1, 2), y64.grad))
print("dmem", e((da + db), m64.grad[0]))
# check pieces: dmem_a alone = sum_px gyn[px][k] P[px][s]
da_ref = torch.einsum("npk,nps->ks", gyn.double().view(N, -1, k), Pr.transpose(1, 2))
print("dmem_a", e(da, da_ref))
gP_ref = torch.einsum("npk,ks->nps", gyn.double().view(N, -1, k), mem.detach().double()[0])
print("gP", e(gP.buf.view(N, -1, S), gP_ref))
