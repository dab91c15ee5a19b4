"""world ranks (2, 4 or 8) on ONE GPU (gloo for the handle exchange): the IPC-mapped one-shot and two-shot
all-reduces must equal the sum of every rank's tensor, and the one-shot all-gather the rank-major
concatenation, repeatedly, at mixed sizes and inside a HIP graph."""
import os

import torch


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    # every rank's spinning workgroups must fit on the ONE shared GPU together (8 x 32 x 512 threads), and a
    # barrier that still never completes errors out in seconds instead of hanging the test
    os.environ.setdefault("SHAI_P2P_MAX_BLOCKS", str(256 // world))
    os.environ.setdefault("SHAI_P2P_TIMEOUT_S", "10")
    import torch.distributed as dist
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    from shai_amd.parallel.comm import P2PAllReduce
    ar = P2PAllReduce(None, max_bytes=8 << 20, one_shot_max=512 << 10)
    # one-shot sizes, then two-shot (reduce-scatter + all-gather) sizes incl. an uneven segmentation
    for n in (8, 4096 * 32, 1 << 18, 1 << 19, (3 << 20) + 8, 4 << 20):
        for it in range(3):
            torch.manual_seed(100 * it + n)
            full = [torch.randn(n, device="cuda").bfloat16() for _ in range(world)]
            x = full[rank].clone()
            ar.all_reduce(x)
            torch.cuda.synchronize()
            want = sum(f.float() for f in full)
            err = ((x.float() - want).abs().max() / want.abs().max()).item()
            assert err < 2e-2, (n, it, err)
            dist.barrier()
    # all-gather (vocab-parallel logits: [B, V / world] shards -> [world * B, V / world] rank-major)
    for rows, cols in ((1, 8), (64, 4096), (3, 1000), (64, 16032)):
        torch.manual_seed(rows * 7 + cols)
        full = [torch.randn(rows, cols, device="cuda").bfloat16() for _ in range(world)]
        out = torch.empty(world * rows, cols, device="cuda", dtype=torch.bfloat16)
        assert ar.can_gather(rows * cols * 2) == ((rows * cols * 2) % 16 == 0)
        if ar.can_gather(rows * cols * 2):
            ar.all_gather_into(out, full[rank])
            torch.cuda.synchronize()
            assert torch.equal(out, torch.cat(full, 0)), (rows, cols)
        dist.barrier()
    # graph replay
    x = torch.ones(4096, device="cuda").bfloat16() * (rank + 1)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        ar.all_reduce(x.clone())
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    y = x.clone()
    with torch.cuda.graph(g):
        ar.all_reduce(y)
    for it in range(3):
        y.copy_(x)
        dist.barrier()
        g.replay()
        torch.cuda.synchronize()
        want = world * (world + 1) / 2
        assert torch.allclose(y.float(), torch.full_like(y.float(), want)), y[:4]
        dist.barrier()
    assert not ar.error()
    dist.barrier()
    ar.close()
    dist.destroy_process_group()
