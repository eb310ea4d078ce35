"""Worker for test_rccl_backend_executes (torch.distributed.run, ONE rank on the one GPU,
backend "nccl" = RCCL): the collective calls the data-parallel path makes
(dgvcc_amd/dist.py, dgvcc_amd/syncbn.py) -- the blocking all-reduce of a flat fp32 gradient,
bucket all-reduces with async_op=True on a side stream (OverlapReducer), broadcast of
parameters/buffers, all_gather of a SyncBN statistics row, barrier and a MAX all-reduce of the
elapsed time -- run through RCCL with the shapes and dtypes they use.  One rank cannot exercise
the xGMI transport (two ranks on one GPU are refused by RCCL); the driver's 8-GPU bench does."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    g = torch.Generator(device=dev).manual_seed(5)
    flat = torch.randn(25_000_003, device=dev, generator=g)  # ~100 MB, odd length
    ref = flat.clone()
    dist.all_reduce(flat)
    assert torch.equal(flat, ref)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        hs = [dist.all_reduce(flat[a:a + 4_000_000], async_op=True) for a in range(0, flat.numel(), 4_000_000)]
    for h in hs:
        h.wait()
    torch.cuda.current_stream().wait_stream(side)
    assert torch.equal(flat, ref)
    for t in (torch.randn(64, 3, 3, 3, device=dev), torch.zeros(1, dtype=torch.long, device=dev),
              torch.ones(512, device=dev)):
        c = t.clone()
        dist.broadcast(c, 0)
        assert torch.equal(c, t)
    row = torch.randn(4, 512, device=dev)
    out = [torch.empty_like(row)]
    dist.all_gather(out, row.contiguous())
    assert torch.equal(out[0], row)
    glob = torch.randn(4, 256, device=dev)
    g0 = glob.clone()
    dist.all_reduce(glob)
    assert torch.equal(glob, g0)
    dist.barrier()
    t = torch.tensor([1.25], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert t.item() == 1.25
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("OK rccl")


if __name__ == "__main__":
    main()
