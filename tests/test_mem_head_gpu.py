"""Memory read folded into the density head (dg_softmax_head_*, dg_mem_head_*; memread.hip).

The reference computes y_new = bmm(mem, softmax(logits)) and then den_head = ReLU(conv1x1(y_new))
(models/models.py:116-125, 112-114, 328-329).  The HIP path never forms y_new: d = act(v . P + b)
with v = mem^T w, and the backward uses the rank-1 structure of g_ynew.  Checked here:
* the kernels against float64 torch autograd of the reference's formulas (logits given), for
  one view, two views with the JSD-MSE (DGModel_memadd/final) and with the KL-JSD
  (models2.DensityRegressorM), and the head-only backward (DensityRegressorM raw=False);
* a final-mode train step on the fused path against the materialised-readout path
  (engine.MEM_HEAD_FUSED = False), same weights and frames.
"""
import os
import tempfile

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _ref(l1, l2, mem, w, b, gd1, gd2, coef, loss_kind):
    """float64 autograd of the reference ops; logits l [B, C, HW] (slot dim 1)."""
    l1 = l1.double().requires_grad_(True)
    l2 = l2.double().requires_grad_(True) if l2 is not None else None
    mem = mem.double().requires_grad_(True)
    w = w.double().requires_grad_(True)
    b = b.double().requires_grad_(True)

    def head(P, B, HW):
        ynew = torch.bmm(mem.unsqueeze(0).expand(B, -1, -1), P)  # [B, k, HW]
        return F.relu(torch.einsum("k,bkp->bp", w, ynew) + b)

    B, C, HW = l1.shape
    p1 = F.softmax(l1, 1)
    d1 = head(p1, B, HW)
    tot = (d1 * gd1.double()).sum()
    d2 = loss = None
    if l2 is not None:
        p2 = F.softmax(l2, 1)
        d2 = head(p2, B, HW)
        tot = tot + (d2 * gd2.double()).sum()
        if loss_kind == 1:
            loss = F.mse_loss(p1, p2)
        else:
            pm = (p1 + p2) / 2
            loss = 0.5 / HW * (F.kl_div(F.log_softmax(l1, 1), pm, reduction="batchmean")
                               + F.kl_div(F.log_softmax(l2, 1), pm, reduction="batchmean"))
        tot = tot + coef * loss
    tot.backward()
    return dict(p1=p1.detach(), d1=d1.detach(), d2=None if d2 is None else d2.detach(),
                loss=None if loss is None else loss.item(), gl1=l1.grad, gl2=None if l2 is None else l2.grad,
                gmem=mem.grad, gw=w.grad, gb=b.grad)


@pytest.mark.parametrize("nv,loss_kind,C", [(1, 0, 1024), (2, 1, 1024), (2, 2, 1024), (2, 1, 512)])
def test_softmax_head_kernels_match_reference(dev, nv, loss_kind, C):
    from dgvcc_amd import kernels as K
    B, HW, k = 2, 96, 256
    g = torch.Generator().manual_seed(11 + nv + loss_kind)
    l1 = torch.randn(B, C, HW, generator=g) * 2
    l2 = l1 + 0.3 * torch.randn(B, C, HW, generator=g) if nv == 2 else None
    mem = torch.randn(k, C, generator=g)
    w = torch.randn(k, generator=g) * 0.05
    b = torch.tensor([0.02])  # ReLU active on roughly half the pixels
    gd1 = torch.randn(B, HW, generator=g)
    gd2 = torch.randn(B, HW, generator=g)
    coef = 3.0
    ref = _ref(l1, l2, mem, w, b, gd1, gd2, coef, loss_kind)
    assert 0.2 < (ref["d1"] > 0).double().mean().item() < 0.8

    M = B * HW
    rows = lambda t: t.permute(0, 2, 1).reshape(M, C).contiguous().to(dev)  # NHWC rows [px][slot]
    L1 = rows(l1)
    L2 = rows(l2) if nv == 2 else None
    memd, wd, bd = mem.to(dev), w.to(dev), b.to(dev)
    v = torch.empty(C, device=dev)
    K.call("dg_mem_head_vec", K.ptr(memd), K.ptr(wd), k, C, K.ptr(v), K.stream())
    P1, P2 = torch.empty(M, C, device=dev), torch.empty(M, C, device=dev)
    yh1, yh2 = torch.empty(M, device=dev), torch.empty(M, device=dev)
    lo = torch.empty((), device=dev)
    work = torch.empty(K.query("dg_mem_head_workspace", M, C) // 4 + 1, device=dev)
    K.call("dg_softmax_head_fwd", 0, nv, loss_kind, K.ptr(L1), K.ptr(L2), M, C, K.ptr(v), K.ptr(bd), 1,
           K.ptr(P1), K.ptr(P2) if nv == 2 else None, K.ptr(yh1), K.ptr(yh2) if nv == 2 else None,
           K.ptr(lo) if loss_kind else None, K.ptr(work), K.stream())
    G1, G2 = gd1.reshape(M).to(dev), gd2.reshape(M).to(dev)
    GL1, GL2 = torch.empty_like(P1), torch.empty_like(P2)
    cf = torch.tensor([coef], device=dev)
    nw = K.amax_words(C)  # f32: operand maxima with channels (slots) per view, nw words each
    am = torch.full((2 * nw,), -1.0, device=dev)
    K.call("dg_softmax_head_bwd", 0, nv, loss_kind, K.ptr(P1), K.ptr(P2) if nv == 2 else None, M, C, K.ptr(v), 1,
           K.ptr(yh1), K.ptr(yh2) if nv == 2 else None, K.ptr(G1), K.ptr(G2) if nv == 2 else None,
           K.ptr(cf) if loss_kind else None, K.ptr(GL1), K.ptr(GL2) if nv == 2 else None, K.ptr(work), K.ptr(am),
           K.stream())
    dmem, gw, gb = torch.empty(k, C, device=dev), torch.empty(k, device=dev), torch.empty(1, device=dev)
    K.call("dg_mem_head_grads", K.ptr(work), M, C, K.ptr(memd), K.ptr(wd), k, K.ptr(dmem), K.ptr(gw), K.ptr(gb),
           K.stream())
    torch.cuda.synchronize()
    back = lambda t: t.reshape(B, HW, C).permute(0, 2, 1)
    assert _rel(back(P1.cpu()), ref["p1"]) < 1e-6
    assert _rel(yh1.view(B, HW), ref["d1"]) < 1e-5
    if nv == 2:
        assert _rel(yh2.view(B, HW), ref["d2"]) < 1e-5
        assert abs(lo.item() - ref["loss"]) <= 1e-5 * abs(ref["loss"])
    assert _rel(back(GL1.cpu()), ref["gl1"]) < 1e-4
    # the pass's operand maxima of gL (the logits GEMMs' f16 x3 scales): tensor word, then one per slot
    assert am[0].item() == GL1.abs().max().item()
    assert torch.equal(am[1:1 + C], GL1.abs().amax(dim=0))
    if nv == 2:
        assert _rel(back(GL2.cpu()), ref["gl2"]) < 1e-4
        assert am[nw].item() == GL2.abs().max().item()
        assert torch.equal(am[nw + 1:nw + 1 + C], GL2.abs().amax(dim=0))
    # dmem here is the readout's share only (the logits' share comes from the logits GEMM)
    assert _rel(dmem, ref["gmem"]) < 1e-5
    assert _rel(gw, ref["gw"]) < 1e-5
    assert abs(gb.item() - ref["gb"].item()) <= 1e-5 * max(1.0, abs(ref["gb"].item()))

    # head-only backward (DensityRegressorM.forward(raw=False)): no logit gradients, same gw/gb
    K.call("dg_softmax_head_bwd", 0, nv, loss_kind, K.ptr(P1), K.ptr(P2) if nv == 2 else None, M, C, K.ptr(v), 1,
           K.ptr(yh1), K.ptr(yh2) if nv == 2 else None, K.ptr(G1), K.ptr(G2) if nv == 2 else None, None, None,
           None, K.ptr(work), None, K.stream())
    gw2, gb2 = torch.empty_like(gw), torch.empty_like(gb)
    K.call("dg_mem_head_grads", K.ptr(work), M, C, K.ptr(memd), K.ptr(wd), k, None, K.ptr(gw2), K.ptr(gb2),
           K.stream())
    torch.cuda.synchronize()
    assert torch.equal(gw2, gw) and torch.equal(gb2, gb)


def test_softmax_head_eval_without_probabilities(dev):
    """P = NULL (eval forward): the head output is the same bits as with P stored."""
    from dgvcc_amd import kernels as K
    M, C, k = 300, 1024, 256
    g = torch.Generator().manual_seed(5)
    L = (torch.randn(M, C, generator=g) * 2).to(dev)
    v = torch.randn(C, generator=g).to(dev)
    b = torch.tensor([0.1], device=dev)
    ya, yb = torch.empty(M, device=dev), torch.empty(M, device=dev)
    P = torch.empty(M, C, device=dev)
    K.call("dg_softmax_head_fwd", 0, 1, 0, K.ptr(L), None, M, C, K.ptr(v), K.ptr(b), 1, K.ptr(P), None, K.ptr(ya),
           None, None, None, K.stream())
    K.call("dg_softmax_head_fwd", 0, 1, 0, K.ptr(L), None, M, C, K.ptr(v), K.ptr(b), 1, None, None, K.ptr(yb),
           None, None, None, K.stream())
    torch.cuda.synchronize()
    assert torch.equal(ya, yb)
    ref = F.relu(F.softmax(L.double().cpu(), 1) @ v.double().cpu() + 0.1)
    assert _rel(ya, ref) < 1e-6


@pytest.mark.parametrize("name,mode", [("DGModel_final", "final"), ("DGModel_memadd", "add"),
                                       ("DGModel_mem", "base"), ("DGModel_memcls", "cls")])
def test_fused_head_step_matches_materialised_readout(dev, name, mode):
    from oracle import dg_oracle as O
    from dgvcc_amd import engine as E
    from dgvcc_amd.models import models as MM
    kw = dict(pretrained=False, den_dropout=0.0)
    if "cls" in name or name == "DGModel_final":
        kw["cls_dropout"] = 0.0
    runs = []
    for fused in (True, False):
        E.MEM_HEAD_FUSED = fused
        try:
            model = getattr(MM, name)(**kw)
            sd0 = O.seeded_state_dict(model.state_dict())
            model.load_state_dict(sd0)
            model = model.to(dev).set_precision("fp32").train()
            batch = O.synthetic_batch(2, 64, 64, seed=77)
            from dgvcc_amd.trainers.dgtrainer import DGTrainer
            from dgvcc_amd.losses import MSELoss
            with tempfile.TemporaryDirectory() as td:
                cwd = os.getcwd()
                os.chdir(td)
                try:
                    torch.manual_seed(3)
                    tr = DGTrainer(2112, "t", dev, 1000, 10000, mode)
                    opt = torch.optim.SGD(model.parameters(), lr=0.0)
                    loss = tr.train_step(model, MSELoss(), opt, batch, 0)
                finally:
                    os.chdir(cwd)
            runs.append((loss, {n: p.grad.detach().cpu().clone() for n, p in model.named_parameters()
                                if p.grad is not None}))
        finally:
            E.MEM_HEAD_FUSED = True
    (la, ga), (lb, gb) = runs
    assert abs(la - lb) <= 1e-5 * abs(lb), (la, lb)
    assert ga.keys() == gb.keys()
    worst = max(_rel(ga[n], gb[n]) for n in gb if gb[n].norm() > 0)
    assert worst < 1e-3, worst
    for n in [n for n in ("mem", "den_head.0.conv.weight", "den_head.0.conv.bias") if n in gb]:
        assert _rel(ga[n], gb[n]) < 1e-4, (n, _rel(ga[n], gb[n]))
