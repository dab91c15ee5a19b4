"""Skinny (decode-shaped, M <= 64) streaming GEMM kernel vs fp32 PyTorch."""
import pytest
import torch

from shai_amd import ops

pytestmark = pytest.mark.gpu
SKINNY = 1000
SKINNY_FIX = 1100


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


@pytest.mark.parametrize("M,N,K", [(1, 4096, 4096), (7, 6144, 4096), (32, 4096, 14336), (32, 28672, 4096),
                                   (16, 1024, 512), (32, 32768, 4096), (3, 96, 64), (33, 4096, 4096),
                                   (48, 6144, 4096), (64, 28672, 4096), (64, 4096, 14336), (64, 96, 64)])
def test_skinny_plain(cuda, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    r = torch.randn(M, N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, b, residual=r, force_cfg=SKINNY)
    want = x.float() @ w.float().t() + b.float() + r.float()
    assert _rel(out, want) < 1e-2


@pytest.mark.parametrize("act,M", [("silu", 32), ("gelu_tanh", 32), ("silu", 64), ("gelu_tanh", 40)])
def test_skinny_glu_and_act(cuda, act, M):
    N, K = 2 * 2048, 4096
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, act=act, glu=True, force_cfg=SKINNY)
    y = x.float() @ w.float().t()
    f = torch.nn.functional.silu if act == "silu" else (lambda t: torch.nn.functional.gelu(t, approximate="tanh"))
    assert _rel(out, y[:, 0::2] * f(y[:, 1::2])) < 1e-2
    out2 = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out2, act=act, force_cfg=SKINNY)
    assert _rel(out2, f(y)) < 1e-2


@pytest.mark.parametrize("fix", [False, True])
@pytest.mark.parametrize("kg", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("M,N,K,rms", [(32, 4096, 4096, False), (64, 4096, 14336, False), (17, 6144, 4096, True),
                                       (64, 28672, 4096, True), (40, 2080, 4096, False)])
def test_skinny_k_groups(cuda, fix, kg, M, N, K, rms):
    """Every K-group count the tuner may pick, with the separate fold (force_cfg = 1000 + kg) and the
    in-kernel last-arriver fixup (1100 + kg), incl. the folded-RMSNorm epilogue and a ragged last tile."""
    torch.manual_seed(kg + M)
    x = (torch.randn(M, K, device=cuda) * 2).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, b, force_cfg=(SKINNY_FIX if fix else SKINNY) + kg, rms_eps=1e-5 if rms else -1.0)
    xf = x.float()
    if rms:
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    assert _rel(out, xf @ w.float().t() + b.float()) < 1e-2


@pytest.mark.parametrize("rms", [False, True])
def test_skinny_fixup_bitwise_deterministic(cuda, rms):
    """The in-kernel split-K fixup sums the K-group slabs in group order whichever group arrives last, so
    repeated launches are bitwise identical (seeded sampling downstream depends on it)."""
    M, N, K = 64, 6144, 4096
    torch.manual_seed(7)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    outs = []
    for _ in range(12):
        out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        ops.gemm_into(x, w, out, force_cfg=SKINNY_FIX + 8, rms_eps=1e-5 if rms else -1.0)
        outs.append(out)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


def test_skinny_graph_replay_rearms_tickets(cuda):
    """Split-K fixup tickets must re-arm so graph replays stay correct."""
    M, N, K = 48, 1024, 8192   # few tiles, long K -> several K groups (two 32-row X groups)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, force_cfg=SKINNY_FIX + 8)  # eager first: allocates tickets
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.gemm_into(x, w, out, force_cfg=SKINNY_FIX + 8)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(3):  # back-to-back launches reuse the same tickets
            ops.gemm_into(x, w, out, force_cfg=SKINNY_FIX + 8)
    for i in range(5):
        x.copy_(torch.randn(M, K, device=cuda).bfloat16())
        g.replay()
        torch.cuda.synchronize()
        assert _rel(out, x.float() @ w.float().t()) < 1e-2, i


def test_autotuned_decode_shapes(cuda):
    """The tuner may pick skinny or a tile config; either way results are right."""
    for M, N, K in [(32, 6144, 4096), (32, 4096, 4096), (32, 28672, 4096), (32, 4096, 14336), (64, 6144, 4096),
                    (64, 4096, 14336)]:
        x = torch.randn(M, K, device=cuda).bfloat16()
        w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
        y = ops.linear(x, w)
        assert _rel(y, x.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("M,N,K", [(32, 6144, 4096), (5, 4096, 4096), (32, 28672, 4096), (64, 512, 1024),
                                   (64, 6144, 4096), (48, 28672, 4096), (96, 512, 1024)])
def test_folded_rmsnorm_linear(cuda, M, N, K):
    """linear(x, W * diag(g), rms_eps) == rmsnorm(x, g) @ W^T (fused in the skinny kernel for M <= 64,
    explicit unweighted norm + GEMM otherwise)."""
    from shai_amd.ops import reference as ref
    x = (torch.randn(M, K, device=cuda) * 3).bfloat16()
    g = (1 + 0.2 * torch.randn(K, device=cuda)).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    wf = (w.float() * g.float()[None]).bfloat16()
    glu = N == 28672
    y = ops.linear(x, wf, act="silu" if glu else None, glu=glu, rms_eps=1e-5)
    xn = ref.rmsnorm(x.float(), g.float(), 1e-5)[0]
    want = xn @ w.float().t()
    if glu:
        want = want[:, 0::2] * torch.nn.functional.silu(want[:, 1::2])
    assert _rel(y, want) < 2e-2


def test_rope_qkv_cache(cuda):
    from shai_amd.ops import reference as ref
    T, H, Hk, D, nb = 37, 8, 2, 128, 6
    qkv = torch.randn(T, (H + 2 * Hk) * D, device=cuda).bfloat16()
    pos = torch.randint(0, 300, (T,), device=cuda, dtype=torch.int32)
    ang = torch.rand(512, D // 2, device=cuda) * 3
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    slots = torch.randperm(nb * 64, device=cuda)[:T].int()
    slots[3] = -1
    kc = torch.zeros(nb, Hk, 64, D, device=cuda).bfloat16()
    vc = torch.zeros_like(kc)
    kc2, vc2, qkv2 = kc.clone().cpu(), vc.clone().cpu(), qkv.clone().cpu()
    ops.rope_qkv_cache(qkv, pos, cos, sin, kc, vc, slots, H, Hk)
    q = qkv2[:, :H * D].view(T, H, D)
    k = qkv2[:, H * D:(H + Hk) * D].view(T, Hk, D)
    v = qkv2[:, (H + Hk) * D:].view(T, Hk, D)
    ref.rope(q, pos.cpu(), cos.cpu(), sin.cpu(), D, True)
    ref.rope(k, pos.cpu(), cos.cpu(), sin.cpu(), D, True)
    ref.kv_write(k, v, kc2, vc2, slots.cpu())
    assert _rel(qkv[:, :H * D], qkv2[:, :H * D]) < 1e-2
    assert _rel(kc, kc2) < 1e-2 and torch.equal(vc.cpu(), vc2)


def test_fused_sampler_distribution(cuda):
    """Fused top-k/top-p sampler: greedy rows exact; sampled tokens follow the truncated distribution."""
    from shai_amd.engines.llm import sample
    torch.manual_seed(0)
    B, V = 4, 32768
    logits = torch.randn(B, V, device=cuda) * 2
    logits[0, 123] = 50.0
    temps = torch.tensor([0.0, 0.7, 1.0, 0.7], device=cuda)
    tk = torch.tensor([50, 50, 5, 0], device=cuda)
    tp = torch.tensor([0.9, 0.9, 1.0, 0.5], device=cuda)
    g = torch.Generator(device=cuda)
    g.manual_seed(1)
    counts = torch.zeros(B, V)
    for _ in range(400):
        t = sample(logits.bfloat16(), temps, tk, tp, g, all_greedy=False).cpu()
        counts[torch.arange(B), t] += 1
    assert counts[0, 123] == 400
    lb = logits.bfloat16().float().cpu()
    top5 = lb[2].topk(5).indices
    assert counts[2, top5].sum() == 400                     # top-k 5 respected
    top50 = lb[1].topk(50).indices
    assert counts[1, top50].sum() == 400
    # row 2: empirical vs softmax over top-5 at T=1
    p = torch.softmax(lb[2, top5], 0)
    assert (counts[2, top5] / 400 - p).abs().max() < 0.1


def test_fused_sampler_deterministic_with_ties(cuda):
    """bf16 logits are full of exact ties: the fused sampler keeps the lowest-index tied candidates and
    sorts ties by index, so a fixed uniform always draws the same token, and greedy rows pick the first
    maximal index (torch.argmax)."""
    torch.manual_seed(3)
    B, V = 8, 32768
    logits = (torch.randn(B, V, device=cuda) * 0.5).round().bfloat16()   # few distinct values
    logits[:, 100] = logits.max() + 1
    logits[:, 7] = logits.max()                                          # tied row maxima at 7 and 100
    temps = torch.tensor([0.0, 0.7, 1.0, 0.7, 0.0, 1.3, 0.7, 0.7], device=cuda)
    tk = torch.tensor([1, 50, 40, 1000, 5, 0, 3, 64], device=cuda, dtype=torch.int32)
    tp = torch.tensor([1.0, 0.9, 0.95, 0.9, 1.0, 0.8, 1.0, 0.5], device=cuda)
    u = torch.rand(B, device=cuda)
    outs = []
    for _ in range(10):
        o = torch.empty(B, dtype=torch.int32, device=cuda)
        ops.sample(logits, temps, tk, tp, u, o)
        outs.append(o.cpu())
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    assert outs[0][0].item() == 7 and outs[0][4].item() == 7


def test_fused_sampler_negative_logits(cuda):
    """All-negative bf16 logits (the threshold key's low half is then all ones): top-k candidates are
    exactly the k largest, greedy rows are the argmax."""
    torch.manual_seed(5)
    B, V = 6, 32768
    lb = (torch.randn(B, V, device=cuda) * 2 - 80).bfloat16()
    temps = torch.tensor([0.0, 0.7, 1.0, 0.7, 1.5, 0.0], device=cuda)
    tk = torch.tensor([50, 50, 5, 200, 1000, 1], device=cuda, dtype=torch.int32)
    tp = torch.ones(B, device=cuda)
    lf = lb.float()
    kth = torch.stack([lf[i].topk(int(tk[i])).values[-1] for i in range(B)])
    for it in range(50):
        u = torch.rand(B, device=cuda)
        o = torch.empty(B, dtype=torch.int32, device=cuda)
        ops.sample(lb, temps, tk, tp, u, o)
        picked = lf[torch.arange(B, device=cuda), o.long()]
        assert bool((picked >= kth).all()), it
        assert int(o[0]) == int(lf[0].argmax()) and int(o[5]) == int(lf[5].argmax())


@pytest.mark.parametrize("D,H,Hk", [(128, 32, 8), (64, 8, 2)])
@pytest.mark.parametrize("splits", [1, 3])
def test_fused_decode_rope_attention(cuda, D, H, Hk, splits):
    """decode_attention_rope (RoPE + KV-cache write + paged decode attention in one kernel) equals
    rope_qkv_cache followed by decode_attention: same outputs, same cache contents; padding rows
    (slot -1) write nothing."""
    torch.manual_seed(D + splits)
    ctx = [1, 2, 64, 65, 300, 1000, 1]       # context INCLUDING this step's token; last row is padding
    B, nb = len(ctx), 40
    qkv = torch.randn(B, (H + 2 * Hk) * D, device=cuda).bfloat16()
    ang = torch.rand(1024, D // 2, device=cuda) * 3
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    kc = torch.randn(nb, Hk, 64, D, device=cuda).bfloat16()
    vc = torch.randn(nb, Hk, 64, D, device=cuda).bfloat16()
    maxb = 16
    perm = torch.randperm(nb, device=cuda).int()
    bt = torch.zeros(B, maxb, dtype=torch.int32, device=cuda)
    i = 0
    for b, c in enumerate(ctx):
        n = (c + 63) // 64
        bt[b, :n] = perm[i:i + n]
        i += n
    lens = torch.tensor(ctx, dtype=torch.int32, device=cuda)
    pos = lens - 1
    slots = torch.stack([bt[b, (c - 1) // 64] * 64 + (c - 1) % 64 for b, c in enumerate(ctx)]).int()
    slots[-1] = -1
    kc2, vc2, qkv2 = kc.clone(), vc.clone(), qkv.clone()
    o = ops.decode_attention_rope(qkv, kc, vc, bt, lens, pos, cos, sin, slots, H, Hk, num_splits=splits)
    ops.rope_qkv_cache(qkv2, pos, cos, sin, kc2, vc2, slots, H, Hk)
    want = ops.decode_attention(qkv2[:, :H * D].reshape(B, H, D), kc2, vc2, bt, lens, num_splits=splits)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    assert _rel(o[:-1], want.reshape(B, H * D)[:-1]) < 1e-2


@pytest.mark.parametrize("D,H,Hk", [(128, 32, 8), (64, 8, 2)])
@pytest.mark.parametrize("splits", [1, 3])
def test_decode_attention_with_qkv_fold_in_kernel(cuda, D, H, Hk, splits):
    """decode_attention_rope_qkv (QKV GEMM left as split-K partials, folded with the RMSNorm scale inside the decode
    attention kernel) equals the two-step form -- skinny GEMM with the same K-group count and its fold launch, then
    decode_attention_rope -- bit for bit: same output, same KV-cache contents, padding row writes nothing."""
    torch.manual_seed(7 * D + splits)
    ctx = [1, 2, 64, 65, 300, 1000, 1]
    B, nb, K, eps = len(ctx), 40, 2048, 1e-5
    N = (H + 2 * Hk) * D
    x = torch.randn(B, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    ang = torch.rand(1024, D // 2, device=cuda) * 3
    cos, sin = ang.cos().contiguous(), ang.sin().contiguous()
    kc = torch.randn(nb, Hk, 64, D, device=cuda).bfloat16()
    vc = torch.randn(nb, Hk, 64, D, device=cuda).bfloat16()
    perm = torch.randperm(nb, device=cuda).int()
    bt = torch.zeros(B, 16, dtype=torch.int32, device=cuda)
    i = 0
    for b, c in enumerate(ctx):
        n = (c + 63) // 64
        bt[b, :n] = perm[i:i + n]
        i += n
    lens = torch.tensor(ctx, dtype=torch.int32, device=cuda)
    pos = lens - 1
    slots = torch.stack([bt[b, (c - 1) // 64] * 64 + (c - 1) % 64 for b, c in enumerate(ctx)]).int()
    slots[-1] = -1
    part = ops.gemm_partials(x, w, eps)
    kg = part.numel() // (B * (N + 1))
    assert kg >= 2 and part.numel() == kg * B * (N + 1)
    qkv = torch.empty(B, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, qkv, force_cfg=SKINNY + kg, rms_eps=eps)
    # the partials themselves: fp32 reference fold of the slabs
    slabs = part[:kg * B * N].view(kg, B, N).sum(0)
    rstd = torch.rsqrt(part[kg * B * N:].view(kg, B).sum(0) / K + eps)
    assert _rel((slabs * rstd[:, None]).bfloat16(), qkv) < 1e-3
    kc2, vc2 = kc.clone(), vc.clone()
    o = ops.decode_attention_rope_qkv(x, w, eps, kc, vc, bt, lens, pos, cos, sin, slots, H, Hk, num_splits=splits)
    want = ops.decode_attention_rope(qkv, kc2, vc2, bt, lens, pos, cos, sin, slots, H, Hk, num_splits=splits)
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    assert torch.equal(o[:-1], want[:-1])


def test_skinny_fixup_concurrent_streams_and_many_tiles(cuda):
    """In-kernel split-K fixups running at the same time on two streams (each stream owns its ticket slice),
    many back-to-back launches with tiles * K groups large (448 tiles x 16 groups), and a graph replayed
    while eager launches run on another stream: every output equals the separate-fold form bit for bit."""
    torch.manual_seed(3)
    shapes = [(64, 28672, 4096, 16), (32, 4096, 14336, 16), (64, 6144, 4096, 8)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    jobs = []
    for M, N, K, kg in shapes:
        x = torch.randn(M, K, device=cuda).bfloat16()
        w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
        ref = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        ops.gemm_into(x, w, ref, force_cfg=SKINNY + kg)            # fold form (no tickets)
        jobs.append((x, w, ref, kg))
    torch.cuda.synchronize()
    outs = [[torch.empty_like(j[2]) for _ in range(6)] for j in jobs]
    for rep in range(6):
        for si, s in enumerate(streams):
            with torch.cuda.stream(s):
                for ji, (x, w, ref, kg) in enumerate(jobs):
                    if (ji + si) % 2 == 0 or rep % 2 == 0:
                        ops.gemm_into(x, w, outs[ji][rep], force_cfg=SKINNY_FIX + kg)
    torch.cuda.synchronize()
    for ji, (x, w, ref, kg) in enumerate(jobs):
        for rep in range(6):
            assert torch.equal(outs[ji][rep], ref), (ji, rep)
    # a captured graph (its own ticket slice) replayed concurrently with eager launches on another stream
    x, w, ref, kg = jobs[0]
    gout = torch.empty_like(ref)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ops.gemm_into(x, w, gout, force_cfg=SKINNY_FIX + kg)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(4):
            ops.gemm_into(x, w, gout, force_cfg=SKINNY_FIX + kg)
    eout = torch.empty_like(ref)
    for _ in range(4):
        with torch.cuda.stream(streams[0]):
            g.replay()
        with torch.cuda.stream(streams[1]):
            for _ in range(4):
                ops.gemm_into(x, w, eout, force_cfg=SKINNY_FIX + kg)
    torch.cuda.synchronize()
    assert torch.equal(gout, ref) and torch.equal(eout, ref)


def test_sampler_top_k_zero_uses_full_vocabulary(cuda):
    """top_k <= 0 (no top-k) must sample over the WHOLE vocabulary: with 4096 nearly-equiprobable tokens and a
    uniform near 1 the inverse-CDF draw lands far beyond the fused sampler's 1024-candidate buffer (the engine
    routes such rows to the exact full-vocabulary path); top_k = 50 rows stay within their 50."""
    from shai_amd.engines.llm import sample
    V, B = 32768, 4
    logits = torch.full((B, V), -30.0, device=cuda)
    logits[:, :4096] = -torch.arange(4096, device=cuda).float() * 1e-4   # rank i = token i
    logits = logits.bfloat16()
    temps = torch.ones(B, device=cuda)
    top_k = torch.tensor([0, 0, 50, -1], device=cuda)
    top_p = torch.ones(B, device=cuda)
    u = torch.tensor([0.99, 0.5, 0.99, 0.75], device=cuda)
    toks = sample(logits, temps, top_k, top_p, uniforms=u).cpu().tolist()
    assert toks[0] > 3000 and 1500 < toks[1] < 2600 and toks[2] < 50 and toks[3] > 2500, toks


SKINNY2 = 1200
SKINNY2_DEEP = 1250


@pytest.mark.parametrize("M,N,K", [(64, 6144, 4096), (1, 1088, 512), (48, 4096, 1024), (17, 256, 4160)])
@pytest.mark.parametrize("kg", [1, 2, 4, 8])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("base", [SKINNY2, SKINNY2_DEEP])
def test_skinny2_kernel(cuda, M, N, K, kg, rms, base):
    """Wide skinny kernel (gemv2.hip), 3- and 6-stage rings: 128-row tiles incl. a ragged last tile, M < 64
    rows, a K tail, split-K with the in-kernel fixup, folded RMSNorm -- vs fp32 torch."""
    torch.manual_seed(M * 7 + N + kg)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, b, force_cfg=base + kg, rms_eps=1e-5 if rms else -1.0)
    xf = x.float()
    if rms:
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5)
    assert _rel(out, xf @ w.float().t() + b.float()) < 1e-2


@pytest.mark.parametrize("cfg", [SKINNY2 + 1, SKINNY2 + 4, SKINNY2_DEEP + 1, SKINNY2_DEEP + 8])
def test_skinny2_glu_residual_and_graph(cuda, cfg):
    kg = cfg % 50
    torch.manual_seed(kg)
    M, N, K = 64, 2048, 4096
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (torch.randn(N, K, device=cuda) / K ** 0.5).bfloat16()
    out = torch.empty(M, N // 2, device=cuda, dtype=torch.bfloat16)
    ops.gemm_into(x, w, out, act="silu", glu=True, force_cfg=cfg)
    y = x.float() @ w.float().t()
    want = y[:, 0::2] * torch.nn.functional.silu(y[:, 1::2])
    assert _rel(out, want) < 1e-2
    r = torch.randn(M, N, device=cuda).bfloat16()
    r0 = r.clone()
    ops.gemm_into(x, w, r, residual=r, force_cfg=cfg)          # in place: C aliases the residual
    assert _rel(r, y + r0.float()) < 1e-2
    # graph replay re-arms the tickets
    o2 = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.gemm_into(x, w, o2, force_cfg=cfg)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(3):
            ops.gemm_into(x, w, o2, force_cfg=cfg)
    for _ in range(3):
        x.copy_(torch.randn(M, K, device=cuda).bfloat16())
        g.replay()
        torch.cuda.synchronize()
        assert _rel(o2, x.float() @ w.float().t()) < 1e-2
