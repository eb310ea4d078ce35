"""Bayesian loss: oracle pinned to the reference fixtures (CPU) and the HIP
kernel against both (GPU)."""
import os

import numpy as np
import pytest
import torch

from oracle.bl_oracle import bl_loss

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CASES = ["g96_bg", "g96_nobg", "g32_bg"]


def _case(g, name):
    c_size, stride, sigma, bgr, use_bg = g[name + "__cfg"]
    counts = g[name + "__counts"]
    pts = np.split(g[name + "__points"], np.cumsum(counts)[:-1])
    tg = [np.ones(int(n), np.float32) for n in counts]
    return (int(c_size), int(stride), float(sigma), float(bgr), bool(use_bg), pts, tg,
            g[name + "__st"], g[name + "__dens"], g[name + "__loss"][0], g[name + "__grad"])


@pytest.mark.parametrize("name", CASES)
def test_bl_oracle_matches_reference(name):
    g = dict(np.load(os.path.join(GOLD, "bl.npz")))
    c_size, stride, sigma, bgr, use_bg, pts, tg, st, dens, loss, grad = _case(g, name)
    l, gr = bl_loss(pts, st, tg, dens, c_size, stride, sigma, bgr, use_bg)
    assert abs(l - loss) <= 1e-5 * abs(loss)
    assert np.abs(gr - grad).max() <= 1e-5 * np.abs(grad).max()


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_bl_hip_matches_reference(dev, name):
    from dgvcc_amd.losses.bl import BL
    g = dict(np.load(os.path.join(GOLD, "bl.npz")))
    c_size, stride, sigma, bgr, use_bg, pts, tg, st, dens, loss, grad = _case(g, name)
    crit = BL(sigma, c_size, stride, bgr, use_bg, dev)
    d = torch.from_numpy(dens).to(dev).requires_grad_(True)
    out = crit([torch.from_numpy(p).to(dev) for p in pts], torch.from_numpy(st).to(dev),
               [torch.from_numpy(t).to(dev) for t in tg], d)
    out.backward()
    assert abs(out.item() - loss) <= 1e-4 * abs(loss)
    gg = d.grad.cpu().numpy()
    # softmax over points in f32 vs torch CPU: ~1e-4 relative on the posterior
    assert np.abs(gg - grad).max() <= 3e-4 * np.abs(grad).max()


@pytest.mark.gpu
def test_post_prob_rows_sum_to_one(dev):
    from dgvcc_amd.losses.bl import Post_Prob
    pp = Post_Prob(8.0, 64, 8, 1.0, True, dev)
    pts = [torch.rand(5, 2, device=dev) * 64, torch.zeros(0, 2, device=dev)]
    probs = pp(pts, torch.tensor([64.0, 64.0], device=dev))
    assert probs[1] is None and probs[0].shape == (6, 64)
    assert torch.allclose(probs[0].sum(0), torch.ones(64, device=dev), atol=1e-5)
