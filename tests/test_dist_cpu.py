"""Data-parallel plumbing on CPU with gloo at world sizes 2, 4 and 8: the
flat-gradient average the fused optimizer performs, the initial-weight broadcast, the
overlapped reducer's bucket accounting over two taped views, and the SyncBatchNorm row
gather with unequal per-rank batches (one above 2^24 pixels).  The GPU path uses the same
calls over RCCL; only the merge kernel (dg_bn_part_finalize) is replaced here by its float64
restatement."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from dgvcc_amd import dist as D
    D.init_from_env("gloo")
    try:
        flat = torch.arange(10, dtype=torch.float32) * (rank + 1)
        D.average_flat_(flat)
        lin = torch.nn.Linear(4, 3)
        with torch.no_grad():
            lin.weight.fill_(float(rank))
        D.broadcast_module_(lin)
        from dgvcc_amd import syncbn as SB
        sync_ok = (SB.group_of(torch.nn.BatchNorm2d(4)) is None
                   and SB.group_of(torch.nn.SyncBatchNorm(4)) is dist.group.WORLD)
        # SyncBN backward: the pixel counts travel with the sums (row 3, hi + lo, exact in f32)
        # and add up over ranks holding different batch sizes
        sums = torch.zeros((4, 8))
        M = 12_582_913 if rank == 0 else 3  # > 2^23 pixels on one rank, 3 on the other
        SB._count_row(sums, M)
        dist.all_reduce(sums)
        count_ok = float(sums[3, 0].double() + sums[3, 1].double()) == 12_582_913.0 + 3 * (world - 1)
        # OverlapReducer: a second backward into a bucket whose all-reduce is in flight raises
        ps = [torch.nn.Parameter(torch.zeros(3)), torch.nn.Parameter(torch.zeros(5))]
        red = D.OverlapReducer(bucket_mb=1.0)
        red.attach(torch.zeros(8), ps, [0, 3], ps)
        red.forward_seen()
        red.emit({ps[0]: torch.ones(3), ps[1]: torch.full((5,), float(rank + 1))})
        try:
            red.emit({ps[0]: torch.ones(3)})
            guard_ok = False
        except RuntimeError:
            guard_ok = True
        red.finish()
        avg_ok = red.flat[3:].tolist() == [(world + 1) / 2] * 5
        buckets_ok = _reducer_buckets(D, rank, world)
        rows_ok = _syncbn_rows(SB, rank, world)
        q.put((rank, flat.tolist(), float(lin.weight.detach().sum()), D.world(), D.rank(), sync_ok and count_ok,
               guard_ok and avg_ok, buckets_ok, rows_ok))
    except Exception:  # report instead of leaving the parent waiting on the queue
        import traceback
        q.put((rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _grad(rank, layer, view, n):
    g = torch.Generator().manual_seed(1000 * rank + 10 * layer + view)
    return torch.randn(n, generator=g)


def _reducer_buckets(D, rank, world):
    """Six parameters of one plan in buckets of ~64 B, delivered layer by layer in reverse for two
    taped views, as the FeaturePlan backward does: every bucket is all-reduced exactly once, after
    the second view's delivery of its last parameter, and the flat buffer ends as the rank average
    of the summed views.  A parameter outside the plan splits the buckets and comes back."""
    sizes = [7, 3, 12, 5, 9, 4]
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    other = torch.nn.Parameter(torch.zeros(2))
    params = ps[:3] + [other] + ps[3:]
    offs = [0]
    for p in params[:-1]:
        offs.append(offs[-1] + p.numel())
    red = D.OverlapReducer(bucket_mb=64 / (1 << 20))
    flat = torch.zeros(sum(p.numel() for p in params))
    red.attach(flat, params, offs, ps)
    nb = len(red.buckets)
    red.forward_seen()
    red.forward_seen()
    launched = []
    for view in range(2):
        for li in reversed(range(len(ps))):
            before = sum(red.launched)
            rest = red.emit({ps[li]: _grad(rank, li, view, sizes[li])})
            if rest:
                return False
            launched.append(sum(red.launched) - before)
    # nothing is launched during the first view; the second launches every bucket once
    if sum(launched[:len(ps)]) != 0 or sum(launched) != nb:
        return False
    if not red.finish():
        return False
    for li, p in enumerate(ps):
        want = sum(_grad(r, li, 0, sizes[li]) + _grad(r, li, 1, sizes[li]) for r in range(world)) / world
        if not torch.allclose(p.grad, want, rtol=1e-6, atol=1e-6):
            return False
        i = next(k for k, q in enumerate(params) if q is p)
        if p.grad.data_ptr() != flat[offs[i]:offs[i] + sizes[li]].data_ptr():
            return False
    a = offs[3]
    return bool(flat[a:a + 2].abs().sum() == 0) and nb >= 4


def _rank_rows(rank):
    """(M, mean, M2) per channel of rank `rank`'s batch: unequal pixel counts per rank, and rank 1
    holds more than 2^24 pixels (a synthetic row: its pixels are never materialised)."""
    C = 3
    if rank == 1:
        M = (1 << 24) + 12_345
        mean = torch.tensor([0.25, -1.5, 3.0], dtype=torch.float64)
        var = torch.tensor([2.0, 0.5, 1.25], dtype=torch.float64)
        return M, mean, var * M, None
    M = 1000 + 617 * rank
    g = torch.Generator().manual_seed(77 + rank)
    x = (torch.randn(M, C, generator=g) * (1 + rank) + rank).double()
    return M, x.mean(0), ((x - x.mean(0)) ** 2).sum(0), x


def _chan_merge(rows):
    """float64 restatement of dg_bn_part_finalize's merge over rows [k][3][C] (zero-count rows skipped)."""
    r = rows.double()
    n = r[:, 0].sum(0)
    mean = (r[:, 0] * r[:, 1]).sum(0) / n
    keep = (r[:, 0] > 0).double()
    m2 = (keep * (r[:, 2] + r[:, 0] * (r[:, 1] - mean) ** 2)).sum(0)
    return n, mean, m2 / n


def _syncbn_rows(SB, rank, world):
    import torch.distributed as dist
    M, mean, M2, _ = _rank_rows(rank)
    row = torch.stack([torch.full_like(mean, float(M)), mean, M2]).float()
    rows = SB.gather_rows(row, M, dist.group.WORLD)
    if tuple(rows.shape) != (2 * world, 3, 3):
        return False
    # rank order: rank r's rows at 2r, 2r + 1 and their counts add up to its exact M
    for r in range(world):
        Mr = _rank_rows(r)[0]
        if not bool(((rows[2 * r, 0].double() + rows[2 * r + 1, 0].double()) == float(Mr)).all()):
            return False
    n, gmean, gvar = _chan_merge(rows)
    tot = sum(_rank_rows(r)[0] for r in range(world))
    wmean = sum(_rank_rows(r)[0] * _rank_rows(r)[1] for r in range(world)) / tot
    wm2 = sum(_rank_rows(r)[2] + _rank_rows(r)[0] * (_rank_rows(r)[1] - wmean) ** 2 for r in range(world))
    return (float(n[0]) == float(tot) and torch.allclose(gmean, wmean, rtol=2e-7, atol=1e-7)
            and torch.allclose(gvar, wm2 / tot, rtol=2e-7))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_average_and_broadcast_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000) + 7 * world
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    errs = [r[1] for r in res if len(r) == 2]
    assert not errs, errs[0]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [i * (world + 1) / 2 for i in range(10)]
    for rank, flat, wsum, ws, rk, sync_ok, red_ok, buckets_ok, rows_ok in res:
        assert sync_ok  # SyncBatchNorm layers synchronise over WORLD, BatchNorm2d stays local
        assert red_ok  # the reducer's in-flight guard and its bucket average
        assert flat == pytest.approx(expect)
        assert wsum == 0.0  # rank 0's weights everywhere
        assert ws == world and rk == rank
        assert buckets_ok  # every bucket all-reduced once, after the last view; rank average
        assert rows_ok  # SyncBN rows: rank order, exact counts above 2^24, the global statistics


def test_syncbn_local_without_process_group():
    from dgvcc_amd import syncbn as SB
    assert SB.group_of(torch.nn.SyncBatchNorm(8)) is None  # no process group: a local BatchNorm
    assert SB.group_of(None) is None


def test_bench_launcher_dry_run_world8():
    """bench.py's multi-rank path end to end on CPU: `--gpus 8` without a
    torchrun environment starts torch.distributed.run (launch_ranks), the 8 ranks join a gloo group,
    time a toy step with a blocking all-reduce per step, gather the per-rank step times and exposed
    all-reduce times (bench.dp_attribution), and rank 0 prints one JSON line."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--steps", "3",
                        "--warmup", "0", "--dry-run"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    att = out["config"]["allreduce"]
    assert out["n_gpus"] == 8 and out["dry_run"] and out["config"]["parallelism"] == "dp8"
    assert len(att["step_ms_per_rank"]) == 8 and len(att["exposed_ms_per_rank"]) == 8
    assert 0 < att["step_ms_min"] <= att["step_ms_max"] and att["exposed_ms"] >= 0
    assert att["step_ms_max"] == max(att["step_ms_per_rank"])
