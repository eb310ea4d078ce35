"""Data-parallel plumbing on CPU with gloo, world_size 2: the
flat-gradient average the fused optimizer performs and the initial-weight
broadcast.  The GPU path uses the same calls over RCCL."""
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
        count_ok = float(sums[3, 0].double() + sums[3, 1].double()) == 12_582_916.0
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
        avg_ok = red.flat[3:].tolist() == [1.5] * 5
        q.put((rank, flat.tolist(), float(lin.weight.sum()), D.world(), D.rank(), sync_ok and count_ok,
               guard_ok and avg_ok))
    finally:
        dist.destroy_process_group()


def test_average_and_broadcast_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = [i * 1.5 for i in range(10)]
    for rank, flat, wsum, world, rk, sync_ok, red_ok in res:
        assert sync_ok  # SyncBatchNorm layers synchronise over WORLD, BatchNorm2d stays local
        assert red_ok  # the reducer's in-flight guard and its bucket average
        assert flat == pytest.approx(expect)
        assert wsum == 0.0  # rank 0's weights everywhere
        assert world == 2 and rk == rank


def test_syncbn_local_without_process_group():
    from dgvcc_amd import syncbn as SB
    assert SB.group_of(torch.nn.SyncBatchNorm(8)) is None  # no process group: a local BatchNorm
    assert SB.group_of(None) is None
