"""CPU-only checks: the C-ABI library loads and exports every declared symbol,
argument validation (no GPU needed: invalid calls return before any launch),
drop-in surface (state_dict keys identical to the reference), host logic."""
import json
import os

import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_library_exports_every_header_symbol():
    from dgvcc_amd import _capi
    protos = _capi.parse_header()
    lib = _capi.lib()
    missing = [n for n in protos if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.dg_version() == _capi.header_abi_version() == 8
    assert len(protos) >= 30


def test_library_matches_its_sources():
    """The library carries the content hash of the sources it was built from; the binding
    refuses one that differs, so no test can run a stale binary."""
    from dgvcc_amd import _capi, srchash
    assert _capi.library_hash() == srchash.source_hash()
    assert len(srchash.source_hash()) == 16


def test_adamw_step_runs_zero_numel_params():
    """_step_runs walks parameter indices: a zero-numel parameter (same element offset as its
    neighbour) neither steals nor gets the neighbour's step count."""
    from dgvcc_amd.optim import AdamW
    sizes = [3, 0, 4, 5, 0]
    offs = [0]
    for n in sizes:
        offs.append(offs[-1] + n)
    group = {"_offs": offs, "_steps": [0] * len(sizes)}
    out = AdamW._step_runs(group, [(0, 3)])
    assert group["_steps"] == [1, 1, 1, 0, 0]
    assert out == [(0, 7, 1)]
    out = AdamW._step_runs(group, [(1, 2), (3, 5)])  # the zero-numel param alone, then 3..4
    assert group["_steps"] == [1, 2, 1, 1, 1]
    assert out == [(7, 12, 1)]
    out = AdamW._step_runs(group, [(0, 5)])
    assert group["_steps"] == [2, 3, 2, 2, 2]
    assert out == [(0, 3, 2), (3, 12, 2)]


def test_invalid_arguments_rejected_without_gpu():
    from dgvcc_amd import _capi
    L = _capi.lib()
    # null pointers / bad dtype / unsupported shapes return status codes
    assert L.dg_conv_fwd(0, None, 64, 1, 8, 8, 64, None, 64, 3, 3, 1, None, None, 64, 0, None) == -1
    assert L.dg_conv_fwd(0, 1, 64, 1, 8, 8, 64, 1, 64, 3, 3, 0, None, 1, 64, 0, None) == -2  # pad != R//2
    assert L.dg_conv_fwd(1, 1, 64, 1, 8, 8, 48, 1, 64, 3, 3, 1, None, 1, 64, 0, None) == -2  # C % 64
    assert L.dg_conv_fwd(7, 1, 64, 1, 8, 8, 64, 1, 64, 3, 3, 1, None, 1, 64, 0, None) == -1  # dtype
    assert L.dg_bn_workspace(0, 64) == -1
    assert L.dg_maxpool2_fwd(0, 1, 64, 1, 7, 8, 64, 1, 64, None) == -2  # odd H
    assert L.dg_upsample_fwd(0, None, 1, 1, 1, 1, 1, 2, 0, None, 1, None) == -1


def test_wgrad_workspace_plan():
    from dgvcc_amd import _capi
    L = _capi.lib()
    ws = L.dg_conv_wgrad_workspace(1, 16, 48, 64, 512, 512, 3, 3)
    assert ws > 0 and ws % (512 * 512 * 9 * 4) == 0
    assert L.dg_conv_wgrad_workspace(1, 0, 48, 64, 512, 512, 3, 3) == -1


def test_f32_presplit_workspace_is_caller_owned():
    """The split-math f32 convolutions' pre-split filter planes (3 bf16 planes of the filter) are
    part of the caller's dg_conv_fwd_workspace: the library allocates no device memory."""
    import os
    from dgvcc_amd import _capi
    L = _capi.lib()
    for C, Co, R in ((512, 512, 3), (64, 64, 3), (896, 256, 1)):
        ws = L.dg_conv_fwd_workspace(0, 16, 48, 64, C, Co, R, R)
        assert ws >= Co * R * R * C * 6 and ws % 256 == 0, (C, Co, R, ws)
    assert L.dg_conv_fwd_workspace(0, 0, 48, 64, 64, 64, 3, 3) == -1
    csrc = os.path.join(os.path.dirname(_capi.HEADER), "..", "dgvcc_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".h")):
            src = open(os.path.join(csrc, f)).read()
            assert "hipMalloc" not in src and "hipFree" not in src, f


def test_conv_tile_layout_queries(monkeypatch):
    """Rows of epilogue BN partials per conv launch follow the tile layout the launch will use
    (host logic, no GPU): the 256-channel f32 pre-split forward on 256-pixel tiles where they
    quantise onto the 256 CUs no worse than 192-pixel ones (DGVCC_PSPLIT_TALL), the dgrad-epilogue
    partials always on 192-pixel tiles, the 16-bit 128-channel persistent forward on 384-pixel
    tiles (DGVCC_PERS_WIDE)."""
    from dgvcc_amd import _capi
    L = _capi.lib()
    rows = lambda dt, N, H, W, C, Co: L.dg_conv_stats_rows_ex(dt, N, H, W, C, C, Co, 3, 3)  # noqa: E731
    M = 16 * 192 * 256
    assert rows(0, 16, 192, 256, 256, 256) == M // 256            # 12 rounds of 256 px < 16 of 192 px
    assert rows(0, 16, 48, 64, 512, 512) == 16 * 48 * 64 // 192   # 1/16 scale: 2 rounds either way
    assert L.dg_conv_bnpart_rows_ex(0, 16, 192, 256, 256, 256, 256, 3, 3) == M // 192
    assert rows(1, 16, 384, 512, 128, 128) == 16 * 384 * 512 // 384
    monkeypatch.setenv("DGVCC_PSPLIT_TALL", "0")
    monkeypatch.setenv("DGVCC_PERS_WIDE", "0")
    assert rows(0, 16, 192, 256, 256, 256) == M // 192
    assert rows(1, 16, 384, 512, 128, 128) == 16 * 384 * 512 // 256
    monkeypatch.setenv("DGVCC_PSPLIT_TALL", "2")
    assert rows(0, 16, 48, 64, 512, 512) == 16 * 48 * 64 // 256


def test_f32_stats_rows_need_split_room():
    """with epilogue statistics (part != NULL) on a shape whose rows
    dg_conv_stats_rows_ex reports for the pre-split kernels, a call without room for the planes
    is refused (it would fall back to the 256-pixel kernel and write another row count)."""
    from dgvcc_amd import _capi
    L = _capi.lib()
    for (N, H, W, C, Co) in ((16, 48, 64, 512, 512), (4, 64, 512, 64, 64), (16, 192, 256, 256, 256)):
        ws = L.dg_conv_fwd_workspace(0, N, H, W, C, Co, 3, 3)
        planes = (Co * 9 * C * 6 + 255) // 256 * 256  # the filter planes' room (+ the pre-split x after it)
        assert ws >= planes
        # x, w, y, part: dummy non-null pointers (the call returns before any launch)
        assert L.dg_conv_fwd_ex(0, 8, C, N, H, W, C, 8, Co, 3, 3, 1, None, 8, Co, 0, 8, None, 0, None, None) == -2
        assert L.dg_conv_fwd_ex(0, 8, C, N, H, W, C, 8, Co, 3, 3, 1, None, 8, Co, 0, 8, 8, planes - 256, None, None) == -2


def test_call_raises_on_error():
    from dgvcc_amd import _capi
    with pytest.raises(_capi.DGError):
        _capi.call("dg_bn_apply", 0, None, 0, 0, 0, None, None, 0, None, 0, None, 0, None, None)


@pytest.mark.parametrize("name", ["DGModel_base", "DGModel_mem", "DGModel_memadd", "DGModel_cls",
                                  "DGModel_memcls", "DGModel_final"])
def test_state_dict_keys_match_reference(name):
    from dgvcc_amd.models import models as M
    ref = json.load(open(os.path.join(GOLD, "state_dict_keys.json")))[name]
    mine = [[k, list(v.shape)] for k, v in getattr(M, name)(pretrained=False).state_dict().items()]
    assert mine == ref


def test_divide_img_into_patches_semantics():
    from dgvcc_amd.utils.misc import divide_img_into_patches
    img = torch.arange(1 * 3 * 25 * 37, dtype=torch.float32).view(1, 3, 25, 37)
    patches, nh, nw = divide_img_into_patches(img, 10)
    assert (nh, nw) == (3, 4)
    assert patches[0].shape[-2:] == (10, 10) and patches[-1].shape[-2:] == (5, 7)
    rebuilt = torch.cat([torch.cat(patches[i * nw:(i + 1) * nw], -1) for i in range(nh)], -2)
    assert torch.equal(rebuilt, img)


def test_trainer_rejects_unknown_mode_and_loss(tmp_path):
    from dgvcc_amd.trainers.dgtrainer import DGTrainer
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        tr = DGTrainer(1, "v", "cpu", 1000, 10000, "nope")
        with pytest.raises(ValueError):
            tr.compute_count_loss(torch.nn.L1Loss(), None, None)

        class Opt:
            def zero_grad(self):
                pass

        b = (torch.zeros(1, 3, 16, 16), torch.zeros(1, 3, 16, 16), ((), torch.zeros(1, 1, 16, 16),
                                                                      torch.zeros(1, 1, 1, 1)))
        with pytest.raises(ValueError):
            tr.train_step(None, torch.nn.MSELoss(), Opt(), b, 0)
        assert os.path.isdir(os.path.join("logs", "v"))
    finally:
        os.chdir(cwd)


def test_seeded_generator_quirk():
    from dgvcc_amd.utils.misc import get_seeded_generator
    a = torch.rand(3, generator=get_seeded_generator(5))
    b = torch.rand(3, generator=get_seeded_generator(99))
    assert torch.equal(a, b)  # reference ignores the seed (utils/misc.py:139-142)


def test_no_gpu_means_loud_failure():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dgvcc_amd.utils import dmap_gen
    import numpy as np
    with pytest.raises(RuntimeError):
        dmap_gen.gaussian_filter_density_fixed(np.zeros((8, 8)), np.zeros((1, 2)))
