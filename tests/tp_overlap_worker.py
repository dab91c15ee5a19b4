"""Two ranks on ONE GPU: the fused + overlapped row-parallel output stage (row-slab GEMMs into the IPC staging
slot on the compute stream, each slab's staged reduce + residual epilogue forked onto a side stream) equals the
dense product, eagerly and replayed from a HIP graph; below OVERLAP_MIN_ROWS one staged reduce runs unsplit."""
import os

import torch


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    torch.cuda.set_device(0)
    from shai_amd.parallel import comm
    from shai_amd.parallel.layers import RowParallelLinear
    from shai_amd.parallel.state import init_distributed
    from shai_amd.weights import load_into
    init_distributed("gloo", tp_size=world)
    p2p = comm.P2PAllReduce(None, max_bytes=16 << 20)
    comm.enable_p2p(p2p)
    comm.OVERLAP_MIN_ROWS, comm.OVERLAP_CHUNKS = 256, 4
    g = torch.Generator().manual_seed(11)
    K, N, M = 3072, 3072, 1056                       # Flux 512^2 single-block out-projection shape
    w = (torch.randn(N, K, generator=g) / K ** 0.5).bfloat16()
    x = torch.randn(M, K, generator=g).bfloat16()
    res = torch.randn(M, N, generator=g).bfloat16()
    lin = RowParallelLinear(K, N, bias=False, input_is_parallel=False).cuda()
    load_into(lin, {"weight": w}, strict=True)
    xc, rc = x.cuda(), res.cuda()
    want = (x.float() @ w.float().t() + res.float()).cuda()
    assert comm.overlap_chunks(M) == 4

    def rel(a):
        return ((a.float() - want).norm() / want.norm()).item()

    for _ in range(3):
        c0 = p2p.launch_counts()
        y = lin(xc, residual=rc)
        torch.cuda.synchronize()
        assert rel(y) < 2e-2, rel(y)
        c1 = p2p.launch_counts()
        # 4 slabs of 264 rows x 3072 (1.6 MB each): four staged two-shot reduces, no unfused all-reduce
        assert c1["staged_two_shot"] - c0["staged_two_shot"] == 4, (c0, c1)
        assert c1["two_shot"] == c0["two_shot"] and c1["one_shot"] == c0["one_shot"], (c0, c1)
        dist.barrier()
    # the small-row regime (< OVERLAP_MIN_ROWS): one unsplit staged reduce
    xs, rs = xc[:128], rc[:128]
    c0 = p2p.launch_counts()
    ys = lin(xs, residual=rs)
    torch.cuda.synchronize()
    c1 = p2p.launch_counts()
    assert sum(c1[k] - c0[k] for k in ("staged_one_shot", "staged_two_shot")) == 1, (c0, c1)
    ws = (x[:128].float() @ w.float().t() + res[:128].float()).cuda()
    assert ((ys.float() - ws).norm() / ws.norm()).item() < 2e-2
    dist.barrier()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        lin(xc, residual=rc)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    dist.barrier()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        yg = lin(xc, residual=rc)
    for _ in range(3):
        dist.barrier()
        graph.replay()
        torch.cuda.synchronize()
        assert rel(yg) < 2e-2, rel(yg)
    assert not p2p.error()
    dist.barrier()
    # the DEFAULT slab count (comm.overlap_chunks by rows and bytes) at both Flux sizes, asserted by launch counters:
    # 1056 rows (512^2) -> 2 staged reduces, 4608 rows (1024^2; N = 1536 keeps the message under this group's
    # 16 MiB staging cap) -> 4
    comm.OVERLAP_CHUNKS, comm.OVERLAP_MIN_ROWS = None, 1024
    for Md, Nd, want_slabs in ((1056, 3072, 2), (4608, 1536, 4)):
        gd = torch.Generator().manual_seed(Md)
        wd = (torch.randn(Nd, K, generator=gd) / K ** 0.5).bfloat16()
        xd = torch.randn(Md, K, generator=gd).bfloat16()
        rd = torch.randn(Md, Nd, generator=gd).bfloat16()
        lind = RowParallelLinear(K, Nd, bias=False, input_is_parallel=False).cuda()
        load_into(lind, {"weight": wd}, strict=True)
        assert comm.overlap_chunks(Md, Nd) == want_slabs
        c0 = p2p.launch_counts()
        yd = lind(xd.cuda(), residual=rd.cuda())
        torch.cuda.synchronize()
        c1 = p2p.launch_counts()
        assert c1["staged_two_shot"] - c0["staged_two_shot"] == want_slabs, (Md, c0, c1)
        wantd = (xd.float() @ wd.float().t() + rd.float()).cuda()
        assert ((yd.float() - wantd).norm() / wantd.norm()).item() < 2e-2
        dist.barrier()
        # the generic overlapped slab loop (no staged reduce: GEMM per slab, that slab's unstaged all-reduce +
        # epilogue on the side stream) -- same slab count, same values
        comm.P2P_STAGED = False
        c0 = p2p.launch_counts()
        yg2 = lind(xd.cuda(), residual=rd.cuda())
        torch.cuda.synchronize()
        c1 = p2p.launch_counts()
        comm.P2P_STAGED = True
        assert c1["two_shot"] - c0["two_shot"] == want_slabs, (Md, c0, c1)
        assert c1["staged_two_shot"] == c0["staged_two_shot"], (c0, c1)
        assert ((yg2.float() - wantd).norm() / wantd.norm()).item() < 2e-2
        dist.barrier()
    comm.enable_p2p(None)
    p2p.close()
    dist.destroy_process_group()
