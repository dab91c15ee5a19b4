"""world ranks (2, 4 or 8) on ONE GPU (gloo for the handle exchange): the IPC-mapped one-shot and two-shot
all-reduces -- both reached through the DEFAULT size routing (one-shot <= 256 KiB < two-shot <= capacity) --
must equal the sum of every rank's tensor, the staged (GEMM-into-the-slot) reduce with its fused
bias / AdaLN gate / residual epilogue the fp32 reference, and the one-shot all-gather the rank-major
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
    from shai_amd.parallel import comm
    from shai_amd.parallel.comm import P2PAllReduce
    ar = P2PAllReduce(None)                      # default routing thresholds
    assert ar.one_shot_max == 256 << 10 and ar.max_bytes >= 16 << 20, (ar.one_shot_max, ar.max_bytes)
    c0 = ar.launch_counts()
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
    c1 = ar.launch_counts()
    assert c1["one_shot"] - c0["one_shot"] == 3 * 2 and c1["two_shot"] - c0["two_shot"] == 3 * 4, (c0, c1)
    # staged reduce: each rank's partial is written INTO the staging slot (as the row-parallel GEMM does), then
    # one kernel sums the slots and applies residual + gate[row // rpg] * (sum + bias); one-shot and two-shot
    # sizes, the residual updated in place (Flux's gated residual)
    for rows, cols, rpg, inplace in ((64, 4096, 64, False), (1000, 3072, 250, True), (8, 64, 1, False)):
        torch.manual_seed(rows + cols)
        parts = [torch.randn(rows, cols, device="cuda").bfloat16() for _ in range(world)]
        bias = torch.randn(cols, device="cuda").bfloat16()
        res = torch.randn(rows, cols, device="cuda").bfloat16()
        gfull = torch.randn(rows // rpg, 6 * cols, device="cuda").bfloat16()
        gate = gfull[:, 2 * cols:3 * cols]         # a strided chunk of the AdaLN modulation, as in models/flux.py
        want = res.float() + gate.float().repeat_interleave(rpg, 0) * (sum(p.float() for p in parts) + bias.float())
        stage = ar.staging(rows, cols, torch.device("cuda", 0))
        stage.copy_(parts[rank])
        out = res if inplace else torch.empty_like(res)
        before = ar.launch_counts()
        ar.reduce_staged(out, cols, bias, res, gate, rpg)
        torch.cuda.synchronize()
        err = ((out.float() - want).abs().max() / want.abs().max()).item()
        assert err < 2e-2, (rows, cols, err)
        after = ar.launch_counts()
        key = "staged_two_shot" if rows * cols * 2 > ar.one_shot_max else "staged_one_shot"
        assert after[key] == before[key] + 1, (key, before, after)
        dist.barrier()
    # row slabs of one staged output (the overlapped row-parallel stage): slab i reduced from byte offset
    # r0 * cols * 2 of every rank's slot, the gate indexed from the slab's first row
    rows, cols, rpg = 1000, 3072, 250
    torch.manual_seed(99)
    parts = [torch.randn(rows, cols, device="cuda").bfloat16() for _ in range(world)]
    bias = torch.randn(cols, device="cuda").bfloat16()
    res = torch.randn(rows, cols, device="cuda").bfloat16()
    gate = torch.randn(rows // rpg, 2 * cols, device="cuda").bfloat16()[:, cols:]
    want = res.float() + gate.float().repeat_interleave(rpg, 0) * (sum(p.float() for p in parts) + bias.float())
    stage = ar.staging(rows, cols, torch.device("cuda", 0))
    stage.copy_(parts[rank])
    out = torch.empty_like(res)
    for r0, r1 in ((0, 40), (40, 600), (600, 1000)):     # one-shot and two-shot sized slabs
        ar.reduce_staged(out[r0:r1], cols, bias, res[r0:r1], gate, rpg, row0=r0, slot_off=r0 * cols * 2)
    torch.cuda.synchronize()
    err = ((out.float() - want).abs().max() / want.abs().max()).item()
    assert err < 2e-2, err
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
