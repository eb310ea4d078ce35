"""Gaussian density-map scatter: oracle vs reference fixtures (CPU, bit-exact for
the fixed kernel) and the HIP kernels vs fixtures (GPU)."""
import os

import numpy as np
import pytest
import torch

from oracle.dmap_oracle import dmap_adaptive, dmap_fixed

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_adaptive_oracle_matches_reference():
    g = dict(np.load(os.path.join(GOLD, "dmap_adaptive.npz")))
    H, W = (int(v) for v in g["shape"])
    for name in ("many", "dup", "few"):
        mine = dmap_adaptive(g[name + "__points"], H, W)
        ref = g[name + "__dmap"]
        assert np.abs(mine - ref).max() <= 1e-6 * np.abs(ref).max(), name


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["edge", "empty", "full"])
def test_dmap_fixed_hip(dev, name):
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed
    g = dict(np.load(os.path.join(GOLD, "dmap_fixed.npz")))
    H, W = (int(v) for v in g[name + "__shape"])
    ref = g[name + "__dmap"]
    # default: the tile-reduce kernel sums in point order like the reference -> bit-identical
    mine = gaussian_filter_density_fixed(np.zeros((H, W)), g[name + "__points"])
    assert np.array_equal(mine, ref), np.abs(mine - ref).max()
    # the atomic scatter: order-independent sum vs the reference's point-order sum
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed_batch
    pts = torch.as_tensor(g[name + "__points"]).reshape(-1, 2).to(dev)
    at = gaussian_filter_density_fixed_batch([pts], H, W, deterministic=False)[0].cpu().numpy()
    scale = max(np.abs(ref).max(), 1e-30)
    assert np.abs(at - ref).max() <= 1e-6 * scale
    assert abs(at.sum(dtype=np.float64) - ref.sum(dtype=np.float64)) <= 1e-5 * max(1.0, abs(ref.sum()))


@pytest.mark.gpu
def test_dmap_fixed_tiled_dense_bit_exact_and_stable(dev):
    """QNRF-like dense crowd (4000 points, clustered, many overlapping stamps, some outside
    or on the border, negative coordinates): the deterministic kernel equals the oracle's
    point-order f32 sum bit for bit, twice in a row, for a batch of ragged images."""
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed_batch
    rng = np.random.default_rng(5)
    H, W = 200, 328
    sets = []
    for n in (4000, 0, 37):
        c = rng.uniform([0, 0], [W, H], (max(n // 50, 1), 2))
        p = c[rng.integers(0, len(c), n)] + rng.normal(0, 6, (n, 2))
        p[: n // 40] = rng.uniform([-8, -8], [W + 2, H + 2], (n // 40, 2))
        sets.append(p.astype(np.float32))
    tp = [torch.from_numpy(p).to(dev) for p in sets]
    a = gaussian_filter_density_fixed_batch(tp, H, W).cpu().numpy()
    b = gaussian_filter_density_fixed_batch(tp, H, W).cpu().numpy()
    assert np.array_equal(a, b)
    for i, p in enumerate(sets):
        assert np.array_equal(a[i], dmap_fixed(p, H, W)), i


@pytest.mark.gpu
@pytest.mark.parametrize("sigma_r", [(4.0, 7), (15.0, 4), (2.0, 31)])
def test_dmap_fixed_host_weights(dev, monkeypatch, sigma_r):
    """The launcher's host-formed 1-D weights and 512-point chunks (default) give the same map bit
    for bit as the per-block device weights on 256-point chunks (DGVCC_DMAP_HOSTW=0) and as the
    256-point chunks alone (DGVCC_DMAP_PTS=1), at the reference's sigma 4 / radius 7 and at other
    radii (the weights' length 2r + 1 up to the 63 the kernel holds)."""
    from dgvcc_amd import kernels as K
    sigma, radius = sigma_r
    rng = np.random.default_rng(11)
    H, W = 130, 200
    n = np.array([0, 1100, 3])
    pts = torch.from_numpy(rng.uniform([-4, -4], [W + 3, H + 3], (int(n.sum()), 2)).astype(np.float32)).to(dev)
    offs = torch.tensor([0] + np.cumsum(n).tolist(), dtype=torch.int64, device=dev)
    a = K.dmap_fixed(pts, offs, 3, H, W, sigma=sigma, radius=radius).cpu()
    monkeypatch.setenv("DGVCC_DMAP_PTS", "1")
    c = K.dmap_fixed(pts, offs, 3, H, W, sigma=sigma, radius=radius).cpu()
    monkeypatch.setenv("DGVCC_DMAP_HOSTW", "0")
    b = K.dmap_fixed(pts, offs, 3, H, W, sigma=sigma, radius=radius).cpu()
    assert torch.equal(a, b) and torch.equal(a, c)
    assert a.abs().sum() > 0


@pytest.mark.gpu
def test_dmap_fixed_tiled_overfull_bin(dev):
    """1500 points inside one 16x16 region plus a sparse background: a tile whose hits span
    several 256-point chunks of the image's point list; still bit-identical to the oracle and
    run to run."""
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed_batch
    rng = np.random.default_rng(9)
    H, W = 96, 128
    p = np.concatenate([rng.uniform([40, 40], [56, 56], (1500, 2)), rng.uniform([0, 0], [W, H], (300, 2))])
    p = p[rng.permutation(len(p))].astype(np.float32)
    tp = [torch.from_numpy(p).to(dev)]
    a = gaussian_filter_density_fixed_batch(tp, H, W).cpu().numpy()
    b = gaussian_filter_density_fixed_batch(tp, H, W).cpu().numpy()
    assert np.array_equal(a, b)
    assert np.array_equal(a[0], dmap_fixed(p, H, W))


@pytest.mark.gpu
def test_dmap_fixed_batch_full_size_mass(dev):
    """768x1024 property: interior points integrate to 1 (the normalized stamp)."""
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density_fixed_batch
    g = torch.Generator().manual_seed(0)
    pts = [torch.rand(500, 2, generator=g) * torch.tensor([1000.0, 740.0]) + 12 for _ in range(4)]
    out = gaussian_filter_density_fixed_batch([p.to(dev) for p in pts], 768, 1024)
    sums = out.sum(dim=(1, 2)).double().cpu()
    assert torch.allclose(sums, torch.full((4,), 500.0, dtype=torch.float64), rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["many", "dup", "few"])
def test_dmap_adaptive_hip(dev, name):
    from dgvcc_amd.utils.dmap_gen import gaussian_filter_density
    g = dict(np.load(os.path.join(GOLD, "dmap_adaptive.npz")))
    H, W = (int(v) for v in g["shape"])
    ref = g[name + "__dmap"]
    mine = gaussian_filter_density(np.zeros((H, W)), g[name + "__points"])
    assert np.abs(mine - ref).max() <= 1e-6 * np.abs(ref).max()
