"""Generate the golden fixtures by RUNNING THE REFERENCE (/root/reference) on
seeded synthetic inputs.  Run in the build container (the reference does not
exist on the GPU box):

    python tests/golden/make_golden.py

Outputs tests/golden/*.npz (small: inputs + expected outputs only).  The
reference is imported with the import placeholders of oracle/ref_import.py;
its `.cuda()` calls (models/ISW/cov_settings.py:21,24,66) are made
device-agnostic by patching torch.Tensor.cuda to a no-op for this process.
"""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.ref_import import import_ref  # noqa: E402
from oracle import dg_oracle as O  # noqa: E402

N_SAMPLE = 16


def summarize(prefix, d, out):
    """Full tensors when small; else sampled entries + sums (index seed fixed)."""
    g = torch.Generator().manual_seed(7)
    for k, v in d.items():
        v = v.detach().float().reshape(-1)
        key = prefix + k.replace(".", "__")
        if v.numel() <= 1024:
            out[key] = v.numpy()
        else:
            idx = torch.randint(0, v.numel(), (N_SAMPLE,), generator=g)
            out[key + "@idx"] = idx.numpy()
            out[key + "@val"] = v[idx].numpy()
            out[key + "@sum"] = np.array([v.double().sum().item(), v.double().abs().sum().item()])


def gen_dmap():
    dg = import_ref("utils.dmap_gen")
    rng = np.random.default_rng(0)
    out = {}
    cases = []
    H, W = 96, 128
    edge = np.array([[0, 0], [W - 0.5, H - 0.5], [3.2, H - 0.1], [-0.5, 10], [-3.7, 20.2],
                     [W, 5], [5, H], [W - 1, 0.2], [64.9, 48.1], [64.9, 48.1]], np.float32)
    cases.append(("edge", H, W, np.concatenate([rng.uniform(0, [W, H], (40, 2)), edge]).astype(np.float32)))
    cases.append(("empty", H, W, np.zeros((0, 2), np.float32)))
    cases.append(("full", 768, 1024, rng.uniform(0, [1024, 768], (500, 2)).astype(np.float32)))
    for name, H, W, pts in cases:
        ref = dg.gaussian_filter_density_fixed(np.zeros((H, W)), pts)
        out[f"{name}__points"] = pts
        out[f"{name}__shape"] = np.array([H, W])
        out[f"{name}__dmap"] = ref.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "dmap_fixed.npz"), **out)


def run_ref_step(model_cls, kwargs, mode, B, H, W):
    rm = import_ref("models.models")
    dgt = import_ref("trainers.dgtrainer")
    model = getattr(rm, model_cls)(pretrained=False, **kwargs)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    batch = O.synthetic_batch(B, H, W, seed=2112)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        os.chdir(td)
        try:
            tr = dgt.DGTrainer(seed=2112, version="golden", device="cpu", log_para=1000,
                               patch_size=10000, mode=mode)
            opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
            model.train()
            # capture outputs with a forward hook on the top-level module
            loss = tr.train_step(model, torch.nn.MSELoss(), opt, batch, 0)
        finally:
            os.chdir(cwd)
    grads = {k: p.grad if p.grad is not None else torch.zeros_like(p) for k, p in model.named_parameters()}
    return sd0, batch, loss, grads, model.state_dict()


def gen_train(name, model_cls, kwargs, mode, B=2, H=64, W=64):
    sd0, batch, loss, grads, sd1 = run_ref_step(model_cls, kwargs, mode, B, H, W)
    out = {"loss": np.array([loss], np.float64), "shape": np.array([B, H, W])}
    summarize("grad__", grads, out)
    summarize("post__", {k: v for k, v in sd1.items() if not k.endswith("num_batches_tracked")}, out)
    # forward outputs of a second, separate forward from the same initial weights (no step)
    rm = import_ref("models.models")
    model = getattr(rm, model_cls)(pretrained=False, **kwargs)
    model.load_state_dict(sd0)
    model.train()
    imgs1, imgs2, (pts, dmaps, bmaps) = batch
    with torch.no_grad():
        if mode in ("simple", "base"):
            out["out_d1"] = model(imgs1).numpy()
        elif mode == "add":
            d1, d2, loss_con = model.forward_train(imgs1, imgs2)
            out["out_d1"], out["out_d2"] = d1.numpy(), d2.numpy()
            out["out_loss_con"] = np.array([loss_con.item()])
        elif mode == "cls":
            d1, c1 = model(imgs1, bmaps)
            out["out_d1"], out["out_c1"] = d1.numpy(), c1.numpy()
        else:
            dc1, dc2, c1, c2, c_err, loss_con, _ = model.forward_train(imgs1, imgs2, bmaps)
            out["out_dc1"] = dc1.numpy()
            out["out_dc2"] = dc2.numpy()
            out["out_c1"] = c1.numpy()
            out["out_c2"] = c2.numpy()
            out["out_loss_con"] = np.array([loss_con.item()])
    np.savez_compressed(os.path.join(HERE, f"train_{name}.npz"), **out)


def gen_final_err(B=2, H=64, W=64):
    """DGModel_final(has_err_loss=True).forward_train (models/models.py:298-335): its loss_err =
    F.l1_loss(IN(y_den1), IN(y_den2)) and the parameter gradients of loss_err alone, every
    dropout off, seeded weights and batch -> train_final_err.npz."""
    rm = import_ref("models.models")
    model = rm.DGModel_final(pretrained=False, den_dropout=0.0, cls_dropout=0.0, has_err_loss=True)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model.train()
    imgs1, imgs2, (_pts, _dmaps, bmaps) = O.synthetic_batch(B, H, W, seed=2112)
    dc1, dc2, c1, c2, c_err, loss_con, loss_err = model.forward_train(imgs1, imgs2, bmaps)
    loss_err.backward()
    grads = {k: p.grad if p.grad is not None else torch.zeros_like(p) for k, p in model.named_parameters()}
    out = {"shape": np.array([B, H, W]), "out_loss_err": np.array([loss_err.item()], np.float64),
           "out_loss_con": np.array([loss_con.item()], np.float64), "out_dc1": dc1.detach().numpy()}
    summarize("grad__", grads, out)
    np.savez_compressed(os.path.join(HERE, "train_final_err.npz"), **out)




# ---------------------------------------------------------------------------
# models/models2.py classes: outputs and parameter gradients of a fixed scalar objective
# ---------------------------------------------------------------------------
M2_CASES = {  # name -> (ctor kwargs, [(method, input names)])
    "DensityRegressorBase": ({"pretrained": False}, [("forward", ("img1",))]),
    "DensityRegressor": ({"pretrained": False}, [("forward", ("img1", "bmaps"))]),
    "DensityRegressorBaseCls": ({"pretrained": False}, [("forward", ("img1", "bmaps"))]),
    "DensityRegressorM": ({"pretrained": False}, [("forward", ("img1", "bmaps")),
                                                  ("forward_train", ("img1", "img2", "bmaps"))]),
    "Generator": ({}, [("forward", ("img1",))]),
    "Generator0": ({}, [("forward", ("img1",))]),
}


def _flat_outputs(o):
    if isinstance(o, (tuple, list)):
        return [t for x in o for t in _flat_outputs(x)]
    return [o] if isinstance(o, torch.Tensor) else []


def m2_run(name, method, dtype, B=2, H=64, W=64):
    """Run reference models2.<name>.<method> on the seeded batch with every dropout off
    (module p = 0; forward_train's functional F.dropout2d(., 0.5) patched to identity) and
    back-propagate sum_k <out_k, r_k> for fixed r_k.  Returns (outputs, grads, sd0)."""
    m2 = import_ref("models.models2")
    m2.F.dropout2d = lambda x, p=0.5, training=True, inplace=False: x
    kw, _ = M2_CASES[name]
    model = getattr(m2, name)(**kw)
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    for mod in model.modules():
        if isinstance(mod, torch.nn.Dropout2d):
            mod.p = 0.0
    model.to(dtype).train()
    img1, img2, (pts, dmaps, bmaps) = O.synthetic_batch(B, H, W, seed=2112)
    inp = {"img1": img1.to(dtype), "img2": img2.to(dtype), "bmaps": bmaps.to(dtype)}
    args = [inp[a] for a in dict(M2_CASES[name][1])[method]]
    outs = _flat_outputs(getattr(model, method)(*args))
    g = torch.Generator().manual_seed(99)
    obj = 0
    for o in outs:
        r = torch.randn(o.shape, generator=g, dtype=torch.float64).to(dtype)
        obj = obj + (o * r).sum()
    obj.backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in model.named_parameters()}
    return outs, grads, sd0


def gen_models2():
    """models2 fixtures: the float64 run is the exact math; the fp32 run measures the
    reference's own fp32 error, which sets the test tolerance."""
    for name, (_, methods) in M2_CASES.items():
        out = {}
        for method, _ in methods:
            o64, g64, _ = m2_run(name, method, torch.float64)
            o32, g32, _ = m2_run(name, method, torch.float32)
            for i, (a, b) in enumerate(zip(o64, o32)):
                out[f"{method}__out{i}"] = a.detach().numpy()
                err = (b.double() - a).abs().max().item() / max(a.abs().max().item(), 1e-30)
                out[f"{method}__out{i}__ref32_err"] = np.array([err])
            num = sum(float((g32[k].double() - g64[k]).norm() ** 2) for k in g64)
            den = sum(float(g64[k].norm() ** 2) for k in g64)
            out[f"{method}__grad_ref32_err"] = np.array([(num / max(den, 1e-300)) ** 0.5])
            summarize(f"{method}__grad__", {k: v.double() for k, v in g64.items()}, out)
            out[f"{method}__gradnorm"] = np.array([den ** 0.5])
        np.savez_compressed(os.path.join(HERE, f"models2_{name}.npz"), **out)
        print(name, {k: float(v[0]) for k, v in out.items() if "ref32" in k})


def gen_models2_keys():
    import json
    m2 = import_ref("models.models2")
    out = {}
    for name, (kw, _) in M2_CASES.items():
        out[name] = [[k, list(v.shape)] for k, v in getattr(m2, name)(**kw).state_dict().items()]
    json.dump(out, open(os.path.join(HERE, "models2_state_dict_keys.json"), "w"))


def gen_state_dict_keys():
    """Key order + shapes of every DGModel_* state_dict (checkpoint interchange)."""
    import json
    rm = import_ref("models.models")
    out = {}
    for name in ("DGModel_base", "DGModel_mem", "DGModel_memadd", "DGModel_cls", "DGModel_memcls",
                 "DGModel_final"):
        m = getattr(rm, name)(pretrained=False)
        out[name] = [[k, list(v.shape)] for k, v in m.state_dict().items()]
    json.dump(out, open(os.path.join(HERE, "state_dict_keys.json"), "w"))


def gen_bl():
    """losses/bl.py BL on synthetic inputs: loss and d loss / d pre_density."""
    blm = import_ref("losses.bl")
    rng = np.random.default_rng(3)
    out = {}
    cases = [("g96_bg", 768, 8, 8.0, 1.0, True, [37, 0, 5]),
             ("g96_nobg", 768, 8, 8.0, 1.0, False, [20, 1, 9]),
             ("g32_bg", 32, 1, 4.0, 0.5, True, [12, 3])]
    for name, c_size, stride, sigma, bgr, use_bg, ns in cases:
        G = c_size // stride
        pts = [torch.from_numpy(rng.uniform(0, c_size, (n, 2)).astype(np.float32)) for n in ns]
        st = torch.from_numpy(rng.uniform(c_size * 0.8, c_size * 1.2, len(ns)).astype(np.float32))
        tg = [torch.ones(n) for n in ns]
        dens = torch.from_numpy(rng.uniform(0, 0.02, (len(ns), 1, G, G)).astype(np.float32)).requires_grad_(True)
        loss = blm.BL(sigma, c_size, stride, bgr, use_bg, "cpu")(pts, st, tg, dens)
        loss.backward()
        pre = f"{name}__"
        out[pre + "cfg"] = np.array([c_size, stride, sigma, bgr, float(use_bg)])
        out[pre + "counts"] = np.array(ns)
        out[pre + "points"] = np.concatenate([p.numpy().reshape(-1, 2) for p in pts]) if sum(ns) else np.zeros((0, 2), np.float32)
        out[pre + "st"] = st.numpy()
        out[pre + "dens"] = dens.detach().numpy()
        out[pre + "loss"] = np.array([loss.item()])
        out[pre + "grad"] = dens.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "bl.npz"), **out)




def gen_dmap_adaptive():
    dg = import_ref("utils.dmap_gen")
    rng = np.random.default_rng(11)
    out = {}
    H, W = 64, 80
    for name, pts in [("many", rng.uniform(0, [W, H], (25, 2))),
                      ("dup", np.array([[10.5, 10.5], [10.5, 10.5], [30, 40], [31, 40], [60.2, 5.5]])),
                      ("few", np.array([[5.0, 5.0], [70.0, 60.0]]))]:
        pts = pts.astype(np.float32)
        out[name + "__points"] = pts
        out[name + "__dmap"] = dg.gaussian_filter_density(np.zeros((H, W)), pts).astype(np.float32)
    out["shape"] = np.array([H, W])
    np.savez_compressed(os.path.join(HERE, "dmap_adaptive.npz"), **out)


# ---------------------------------------------------------------------------
# ResNet-50 DG trunks (IBN-b / SW / ISW), SwitchWhiten2d and the ISW loss
# ---------------------------------------------------------------------------
def _patch_offline():
    """The counters hard-code pretrained=True (remote weights) and call .cuda();
    build them with pretrained=False and make .cuda() a no-op for this process."""
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    torch.cuda.current_device = lambda: 0  # only gates a log print (cov_settings.py:79)
    ibn = import_ref("models.ibnnet")
    if not getattr(ibn, "_dg_patched", False):
        f = ibn.resnet50_ibn_b
        ibn.resnet50_ibn_b = lambda pretrained=True, **k: f(pretrained=False, **k)
        ibn._dg_patched = True
    sw = import_ref("models.SW")
    if not getattr(sw, "_dg_patched", False):
        f2 = sw.resnet50
        sw.resnet50 = lambda pretrained=True, **k: f2(pretrained=False, **k)
        sw._dg_patched = True
    R = import_ref("models.ISW.Resnet")
    if not getattr(R, "_dg_patched", False):
        f3 = R.resnet50
        R.resnet50 = lambda pretrained=True, **k: f3(pretrained=False, **k)
        R._dg_patched = True
    isw = import_ref("models.ISW")
    return {"ibn": ibn.IBNCounter_ResNet, "sw": sw.SWCounter_ResNet, "isw": isw.ISWCounter_ResNet}


def gen_sw_op():
    _patch_offline()
    swm = import_ref("models.SW.ops.switchwhiten")
    g = torch.Generator().manual_seed(5)
    out = {}
    m = swm.SwitchWhiten2d(32, num_pergroup=16, sw_type=2, T=5, tie_weight=False, eps=1e-5,
                           momentum=0.9, affine=True)
    with torch.no_grad():
        m.sw_mean_weight.copy_(torch.randn(2, generator=g))
        m.sw_var_weight.copy_(torch.randn(2, generator=g))
        m.weight.copy_(torch.rand(32, generator=g) + 0.5)
        m.bias.copy_(torch.randn(32, generator=g) * 0.1)
        m.running_mean.copy_(torch.randn(2, 16, 1, generator=g) * 0.1)
        a = torch.randn(2, 16, 16, generator=g) * 0.3
        m.running_cov.copy_(a @ a.transpose(1, 2) + torch.eye(16))
    for k, v in m.state_dict().items():
        out["init__" + k] = v.numpy().copy()
    x = (torch.randn(3, 32, 5, 7, generator=g) * 2 + 0.5).requires_grad_(True)
    gy = torch.randn(3, 32, 5, 7, generator=g)
    m.train()
    y = m(x)
    y.backward(gy)
    out["x"] = x.detach().numpy()
    out["gy"] = gy.numpy()
    out["y"] = y.detach().numpy()
    out["gx"] = x.grad.numpy()
    for k, p in m.named_parameters():
        out["grad__" + k] = p.grad.numpy()
    for k in ("running_mean", "running_cov"):
        out["post__" + k] = getattr(m, k).numpy()
    m.eval()
    with torch.no_grad():
        out["y_eval"] = m(x.detach()).numpy()
    np.savez_compressed(os.path.join(HERE, "sw_op.npz"), **out)


def gen_iw_loss():
    _patch_offline()
    iwm = import_ref("models.ISW.instance_whitening")
    cs = import_ref("models.ISW.cov_settings")
    g = torch.Generator().manual_seed(6)
    out = {}
    C = 16
    cm = cs.CovMatrix_ISW(dim=C, relax_denom=2.0, clusters=3)
    eye, rev = cm.get_eye_matrix()
    for r in range(2):  # cal_covstat accumulations (ISW/__init__.py:93-104)
        f = torch.randn(4, C, 6, 5, generator=g)
        f = f + 0.5 * f[:, :1]  # correlated channels
        out[f"cov_in{r}"] = f.numpy()
        fc = torch.bmm(f.view(4, C, -1), f.view(4, C, -1).transpose(1, 2)).div(30 - 1) + 1e-5 * eye
        cm.set_variance_of_covariance(torch.var(fc * rev, dim=0))
    eye, mask, margin, ns = cm.get_mask_matrix()
    out["mask"] = mask.numpy()
    out["num_sensitive"] = np.array([float(ns)])
    f_map = torch.randn(3, C, 7, 4, generator=g)
    f_map = (f_map + 0.3 * f_map[:, 1:2]).requires_grad_(True)
    loss = iwm.instance_whitening_loss(f_map, eye, mask, margin, ns)
    loss.backward()
    out["f_map"] = f_map.detach().numpy()
    out["loss"] = np.array([loss.item()])
    out["grad"] = f_map.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "iw_loss.npz"), **out)


def gen_trunk(kind, B=2, H=64, W=64, dtype=torch.float32):
    """dtype float64 for SW: the fp32 reference's Newton-Schulz backward amplifies
    rounding noise to ~1e-2 in early-layer grads; the float64 run is the exact math."""
    ctors = _patch_offline()
    model = ctors[kind]()
    sd0 = O.seeded_state_dict(model.state_dict())
    model.load_state_dict(sd0)
    model.to(dtype)
    img1, img2, (pts, dmaps, bmaps) = O.synthetic_batch(B, H, W, seed=2112)
    img1, img2, dmaps = img1.to(dtype), img2.to(dtype), dmaps.to(dtype)
    out = {"shape": np.array([B, H, W]), "dtype64": np.array([dtype == torch.float64])}
    if kind == "isw":
        model.eval()  # cal_covstat runs from predict2 during validation (dgtrainer.py:94-100)
        with torch.no_grad():
            model([img1, img2], cal_covstat=True)
        masks = []
        for li, cm in enumerate(model.cov_matrix_layer):
            summarize(f"var{li}", {"": cm.var_matrix / cm.count_var_cov}, out)
            _, mk, _, ns = cm.get_mask_matrix()
            out[f"mask{li}"] = np.packbits(mk.numpy().astype(np.uint8).reshape(-1))
            out[f"ns{li}"] = np.array([float(ns)])
            masks.append(mk)
        model.train()
        cap = {}
        h = model.head.register_forward_hook(lambda mod, inp, o: cap.update(out=o.detach()))  # returns None
        loss1, wt = model(img1, gts=dmaps, apply_wtloss=True)
        h.remove()
        out["out"] = cap["out"].numpy()
        total = loss1 + 0.6 * wt  # dgtrainer.py:196-203 (epoch > 5)
        out["loss1"] = np.array([loss1.item()])
        out["wt_loss"] = np.array([float(wt)])
        total.sum().backward()
    else:
        model.train()
        pred = model(img1)
        out["out"] = pred.detach().float().numpy()
        loss = torch.nn.functional.mse_loss(pred, dmaps * 1000)
        out["loss"] = np.array([loss.item()])
        loss.backward()
    grads = {k: p.grad if p.grad is not None else torch.zeros_like(p)
             for k, p in model.named_parameters()}
    summarize("grad__", grads, out)
    summarize("post__", {k: v for k, v in model.state_dict().items()
                         if not k.endswith("num_batches_tracked")}, out)
    np.savez_compressed(os.path.join(HERE, f"trunk_{kind}.npz"), **out)


def gen_trunk_keys():
    import json
    ctors = _patch_offline()
    out = {k: [[n, list(v.shape)] for n, v in c().state_dict().items()] for k, c in ctors.items()}
    json.dump(out, open(os.path.join(HERE, "trunk_state_dict_keys.json"), "w"))


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["dmap", "base", "final", "bl", "keys", "dmap_adaptive"]
    if "dmap" in which:
        gen_dmap()
    if "base" in which:
        gen_train("simple_base", "DGModel_base", {"den_dropout": 0.0}, "simple")
    if "final" in which:
        gen_train("final", "DGModel_final", {"den_dropout": 0.0, "cls_dropout": 0.0}, "final")
    if "final_err" in which:
        gen_final_err()
    # DGTrainer modes of the ablation configs (configs/ablation/*: base/mem -> 'base',
    # memadd -> 'add', cls/memcls -> 'cls'); every dropout off
    for key, cls_name, kw, mode in [("base_base", "DGModel_base", {"den_dropout": 0.0}, "base"),
                                    ("mem_base", "DGModel_mem", {"den_dropout": 0.0}, "base"),
                                    ("memadd_add", "DGModel_memadd", {"den_dropout": 0.0}, "add"),
                                    ("cls_cls", "DGModel_cls", {"den_dropout": 0.0, "cls_dropout": 0.0}, "cls"),
                                    ("memcls_cls", "DGModel_memcls", {"den_dropout": 0.0, "cls_dropout": 0.0},
                                     "cls")]:
        if "modes" in which or key in which:
            gen_train(key, cls_name, kw, mode)
    if "bl" in which:
        gen_bl()
    if "keys" in which:
        gen_state_dict_keys()
    if "dmap_adaptive" in which:
        gen_dmap_adaptive()
    if "sw_op" in which:
        gen_sw_op()
    if "iw_loss" in which:
        gen_iw_loss()
    for kind in ("ibn", "sw", "isw"):
        if "trunk_" + kind in which:
            gen_trunk(kind, dtype=torch.float64 if kind == "sw" else torch.float32)
    if "models2" in which:
        gen_models2()
    if "models2_keys" in which:
        gen_models2_keys()
    if "trunk_keys" in which:
        gen_trunk_keys()
    print("fixtures written to", HERE)
