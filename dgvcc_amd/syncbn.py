"""SyncBatchNorm over data-parallel ranks on the HIP BN kernels.

The reference's ISW trunk normalises with `nn.SyncBatchNorm` (models/ISW/mynn.py:8-14), which
synchronises its batch statistics as soon as a process group exists; torch's
`nn.SyncBatchNorm.convert_sync_batchnorm(model)` opts any other model in (the DGModel_* VGG16-BN
layers for a strong-scaled jhu_fog2snow run: the configs' batch of 16 split over the ranks with
the BN statistics of all 16).  A BN layer takes this path when its module is an
`nn.SyncBatchNorm` and its process group (default: WORLD) has more than one rank; otherwise the
local kernels run unchanged.

The exchange is the one torch's SyncBatchNorm does, in two small collectives per layer:
  forward   each rank's (n, mean, M2) row [3][C] is all-gathered and merged in rank order
            (Chan, double) by dg_bn_part_finalize -> the global statistics + running-stat update;
  backward  each rank's (sum g', sum g' xhat, sum xhat) [3][C] is all-reduced; the dz
            coefficients come from the global sums over all ranks' pixels, dgamma / dbeta (and
            the conv bias) from this rank's, which the data-parallel gradient average then
            combines like every other parameter gradient.
Rows are f32 [3][C] (at most 6 KB per layer; two per rank in the gather, so that the counts stay exact in
f32 at any batch), so the collectives are latency, not bandwidth.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from . import kernels as K
from ._capi import call, ptr, query, stream


def group_of(bn) -> object | None:
    """The process group to synchronise `bn` over, or None for a local BatchNorm."""
    if not isinstance(bn, nn.SyncBatchNorm):
        return None
    if not (dist.is_available() and dist.is_initialized()):
        return None
    pg = bn.process_group if bn.process_group is not None else dist.group.WORLD
    return pg if dist.get_world_size(pg) > 1 else None


_BATCHES: dict = {}  # id(num_batches_tracked) -> [tensor, owed count]


def bump_batches(bn) -> None:
    """bn.num_batches_tracked += 1 (nn.BatchNorm2d.forward in training), deferred: flush_batches()
    adds every owed count in one torch._foreach_add_ launch instead of one launch per layer
    (a plan forward flushes when it ends; a read of the count flushes first)."""
    t = bn.num_batches_tracked
    ent = _BATCHES.get(id(t))
    if ent is None or ent[0] is not t:
        _BATCHES[id(t)] = [t, 1]
    else:
        ent[1] += 1


def flush_batches() -> None:
    if _BATCHES:
        ents = list(_BATCHES.values())
        _BATCHES.clear()
        torch._foreach_add_([e[0] for e in ents], [e[1] for e in ents])


def _momentum(bn) -> float:
    if bn.momentum is None:
        flush_batches()
        return 1.0 / float(bn.num_batches_tracked.item())
    return float(bn.momentum)


def _all_gather_rows(row: torch.Tensor, pg) -> torch.Tensor:
    w = dist.get_world_size(pg)
    out = [torch.empty_like(row) for _ in range(w)]
    dist.all_gather(out, row.contiguous(), group=pg)
    return torch.stack(out)  # [world][...], rank order


# a rank's (n, mean, M2) row carries its pixel count in f32, exact only below 2^24
_ROW_EXACT_M = 1 << 24


def split_row(row: torch.Tensor, M: int) -> torch.Tensor:
    """This rank's (n, mean, M2) row [3][C] over M pixels as two rows [2][3][C] whose counts are
    exact in f32 at any M < 2^36 (no limit at 2^24 pixels per rank).  Below 2^24 the
    row itself and a zero row (which the Chan merge skips); above, counts M - M % 4096 and
    M % 4096 with the same mean and M2 shared in proportion, which merge back to (M, mean, M2)."""
    two = torch.zeros((2,) + tuple(row.shape), dtype=torch.float32, device=row.device)
    if M < _ROW_EXACT_M:
        two[0] = row
        return two
    lo = M % 4096
    hi = M - lo
    for k, n in ((0, hi), (1, lo)):
        two[k, 0] = float(n)
        two[k, 1] = row[1]
        two[k, 2] = (row[2].double() * (n / M)).float()
    return two


def gather_rows(row: torch.Tensor, M: int, pg) -> torch.Tensor:
    """Every rank's split rows in rank order, [world * 2][3][C] (host logic; the merge is
    dg_bn_part_finalize's)."""
    rows = _all_gather_rows(split_row(row, M), pg)
    return rows.reshape((-1,) + tuple(row.shape))


def finalize_rows(bn, row: torch.Tensor, pg, M: int) -> torch.Tensor:
    """Local (n, mean, M2) row over M pixels -> the global stats [4][C] (mean, invstd, scale, shift)."""
    rows = gather_rows(row, M, pg)
    C = row.shape[1]
    bump_batches(bn)
    return K.bn_part_finalize(rows, rows.shape[0], C, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                              bn.running_var, _momentum(bn), bn.eps)


def row_from_z(z: K.Act) -> torch.Tensor:
    row = torch.empty((3, z.C), dtype=torch.float32, device=z.buf.device)
    work = torch.empty(query("dg_bn_workspace", z.M, z.C) // 4 + 1, dtype=torch.float32, device=z.buf.device)
    call("dg_bn_stats_row", z.dt, z.ptr, z.ld, z.M, z.C, ptr(row), ptr(work), stream())
    return row


def row_from_part(part: torch.Tensor, nblk: int, C: int) -> torch.Tensor:
    row = torch.empty((3, C), dtype=torch.float32, device=part.device)
    work = torch.empty(query("dg_bn_part_workspace", nblk, C) // 4 + 1, dtype=torch.float32, device=part.device)
    call("dg_bn_part_row", ptr(part), nblk, C, ptr(row), ptr(work), stream())
    return row


def fwd_stats(bn, pg, z: K.Act | None = None, part: torch.Tensor | None = None, nblk: int = 0,
              M: int = 0) -> torch.Tensor:
    """Global batch statistics of a synchronised BN layer from this rank's z or its partial rows
    (M: the pixels those rows cover)."""
    row = row_from_part(part, nblk, bn.num_features) if part is not None else row_from_z(z)
    return finalize_rows(bn, row, pg, M if part is not None else z.M)


def _count_row(sums: torch.Tensor, M: int):
    """Row 3 of the sums: this rank's pixel count as hi + lo parts, each exact in f32, so the
    all-reduced row carries the global count even when the ranks' batches differ."""
    lo = M % 4096
    sums[3].zero_()
    sums[3, 0] = float(M - lo)
    sums[3, 1] = float(lo)


def bwd_sums(g: K.Act, z: K.Act, stats, act: int, drop=None, g_pool: K.Act | None = None,
             part: torch.Tensor | None = None, nblk: int = 0) -> torch.Tensor:
    """This rank's BN-backward sums [4][C]: (sum g', sum g' xhat, sum xhat) from (g, z), from the
    pooled gradient g_pool (+ the direct g) with the argmax recomputed from z, or from
    dgrad-epilogue partial rows; row 3 the pixel count (_count_row)."""
    C, dev = z.C, z.buf.device
    sums = torch.empty((4, C), dtype=torch.float32, device=dev)
    _count_row(sums, z.M)
    if part is not None:
        call("dg_bn_part_sums", ptr(part), nblk, C, ptr(sums), stream())
        return sums
    if g_pool is not None:
        work = torch.empty(query("dg_bn_workspace", z.M, C) // 4 + 1, dtype=torch.float32, device=dev)
        call("dg_bn_bwd_pool_sums", z.dt, g_pool.ptr, g_pool.ld, g.ptr if g is not None else None,
             g.ld if g is not None else 0, z.ptr, z.ld, z.N, z.H, z.W, C, ptr(stats[0]), ptr(stats[1]),
             ptr(stats[2]), ptr(stats[3]), act, ptr(drop), ptr(sums), ptr(work), stream())
        return sums
    work = torch.empty(query("dg_bn_workspace", z.M, C) // 4 + 1, dtype=torch.float32, device=dev)
    call("dg_bn_bwd_sums", z.dt, g.ptr, g.ld, z.ptr, z.ld, z.M, C, ptr(stats[0]), ptr(stats[1]), ptr(stats[2]),
         ptr(stats[3]), act, ptr(drop), z.H * z.W, ptr(sums), ptr(work), stream())
    return sums


def bwd_coef(bn, pg, sums: torch.Tensor, M_local: int, stats, dgamma, dbeta, dbias=None) -> torch.Tensor:
    """All-reduce the sums [4][C]; the dz coefficients [3][C] from the global ones over the
    global pixel count (the all-reduced row 3: ranks may hold different batch sizes, as torch's
    SyncBatchNorm allows), dgamma / dbeta / dbias from this rank's."""
    glob = sums.clone()
    dist.all_reduce(glob, group=pg)
    C = sums.shape[1]
    coef = torch.empty((3, C), dtype=torch.float32, device=sums.device)
    call("dg_bn_bwd_finalize_sync", ptr(sums), ptr(glob), M_local, -1, C,
         ptr(bn.weight.detach()), ptr(stats[1]), ptr(dgamma), ptr(dbeta), ptr(dbias), ptr(coef), stream())
    return coef


def bwd_apply(g: K.Act, z: K.Act, stats, act: int, coef, dz: K.Act, drop=None, g_pool: K.Act | None = None):
    am = K._amax_out(dz)
    if g_pool is not None:
        call("dg_bn_bwd_pool_apply_coef", z.dt, g_pool.ptr, g_pool.ld, g.ptr if g is not None else None,
             g.ld if g is not None else 0, z.ptr, z.ld, z.N, z.H, z.W, z.C, ptr(stats[0]), ptr(stats[1]),
             ptr(stats[2]), ptr(stats[3]), act, ptr(drop), ptr(coef), dz.ptr, dz.ld, ptr(am), stream())
    else:
        call("dg_bn_bwd_apply_coef", z.dt, g.ptr, g.ld, z.ptr, z.ld, z.M, z.C, ptr(stats[0]), ptr(stats[1]),
             ptr(stats[2]), ptr(stats[3]), act, ptr(drop), z.H * z.W, ptr(coef), dz.ptr, dz.ld, ptr(am), stream())


def backward(bn, pg, g: K.Act | None, z: K.Act, stats, act: int, dz: K.Act | None, dgamma, dbeta, dbias=None,
             drop=None, g_pool: K.Act | None = None, part: torch.Tensor | None = None, nblk: int = 0):
    """The whole synchronised BN(+ReLU[+pool]) backward; returns the coefficients (dz = None:
    coefficients only, for a fused consumer such as the stem's weight-gradient pass)."""
    sums = bwd_sums(g, z, stats, act, drop=drop, g_pool=g_pool, part=part, nblk=nblk)
    coef = bwd_coef(bn, pg, sums, z.M, stats, dgamma, dbeta, dbias)
    if dz is not None:
        bwd_apply(g, z, stats, act, coef, dz, drop=drop, g_pool=g_pool)
    return coef
