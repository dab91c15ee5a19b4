#!/usr/bin/env python3
"""Kernel microbenchmarks on the GPU: shai kernels vs PyTorch-ROCm library paths
(hipBLASLt GEMM, MIOpen conv, SDPA) on the same random bf16 inputs.

python tools/bench_kernels.py [--only gemm,conv,attn,norm] [--json out.json]
"""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

import shai_amd.ops as ops


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def graph_time(fn, iters=32, reps=5):
    """Seconds per call of fn with the host out of the loop: `iters` calls captured into one HIP graph, the
    replay timed with events (best of `reps`).  For kernels shorter than the host's per-call launch cost."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e-3)
    return best


def rnd(*shape):
    return torch.randn(*shape, device="cuda").to(torch.bfloat16)


def bench_gemm(rows):
    shapes = [(32768, 320, 320), (32768, 2560, 320), (32768, 320, 1280), (8192, 1280, 5120), (4096, 4096, 4096),
              (8192, 8192, 8192), (2048, 12288, 3072), (256, 4096, 4096), (64, 14336, 4096)]
    for M, N, K in shapes:
        a, w = rnd(M, K), rnd(N, K)
        t_s = timeit(lambda: ops.linear(a, w))
        t_t = timeit(lambda: torch.matmul(a, w.t()))
        f = 2 * M * N * K
        rows.append(dict(op="gemm", shape=f"{M}x{N}x{K}", shai_us=t_s * 1e6, torch_us=t_t * 1e6,
                         shai_tflops=f / t_s / 1e12, torch_tflops=f / t_t / 1e12))


def bench_decode(rows):
    """Decode-shaped GEMMs (Mistral-7B TP1, batch M): skinny kernel vs each tile config vs hipBLASLt,
    reported as achieved weight bandwidth."""
    cfgs = int(os.environ.get("SHAI_NUM_CFGS", "5"))
    for M in [int(m) for m in os.environ.get("SHAI_DECODE_M", "1,8,32,64").split(",")]:
        for N, K in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (32768, 4096)]:
            # rotate over enough weight copies to defeat the 256 MB Infinity Cache (decode streams
            # 14.5 GB of weights per token, so every GEMM reads HBM)
            ncopy = max(2, min(16, (768 << 20) // (N * K * 2) + 1))
            a = rnd(M, K)
            ws = [rnd(N, K) * 0.02 for _ in range(ncopy)]
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws[it[0]]
            res = {}
            kgs = (1, 2, 4, 8, 16)
            v1 = [1000] + [1100 + kg for kg in kgs[1:]]
            v2 = [1200 + kg for kg in kgs] + [1250 + kg for kg in kgs]
            for c in list(range(cfgs)) + v1 + v2:
                try:
                    res[c] = timeit(lambda: ops.gemm_into(a, nxt(), out, force_cfg=c), iters=48)
                except Exception as e:  # noqa
                    res[c] = float("nan")
            t_t = timeit(lambda: torch.matmul(a, nxt().t()), iters=48)
            t_tuned = timeit(lambda: ops.linear(a, nxt()), iters=48)
            del ws
            gb = N * K * 2 / 1e9

            def best(keys):
                return min(((res[k], k) for k in keys if res[k] == res[k]), default=(float("nan"), -1))
            s1, s2 = best(v1), best(v2)
            rows.append(dict(op="decode_gemm", shape=f"{M}x{N}x{K}", skinny_us=s1[0] * 1e6, skinny_cfg=s1[1],
                             skinny2_us=s2[0] * 1e6, skinny2_cfg=s2[1], skinny2_TBps=gb / s2[0] / 1e3,
                             best_tile_us=min((res[k] for k in range(cfgs)), default=float("nan")) * 1e6,
                             tuned_us=t_tuned * 1e6, tuned_TBps=gb / t_tuned / 1e3, torch_us=t_t * 1e6,
                             skinny_TBps=gb / s1[0] / 1e3, torch_TBps=gb / t_t / 1e3))


def bench_decode_fp8(rows):
    """Decode GEMMs at M = 1 / 32 / 64: skinny kernel with bf16 vs fp8-e4m3 weights, per K-group
    count, as time and achieved weight bandwidth (bf16-equivalent bytes / time for fp8)."""
    for M in (1, 32, 64):
        for N, K in [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]:
            ncopy = max(2, min(16, (768 << 20) // (N * K * 2) + 1))
            a = rnd(M, K)
            wb = [rnd(N, K) * 0.02 for _ in range(ncopy)]
            w8 = [ops.quantize_fp8_rows(w) for w in wb]
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            it = [0]

            def nxt(lst):
                it[0] = (it[0] + 1) % ncopy
                return lst[it[0]]
            best = {}
            for name in ("bf16", "fp8"):
                for kg in (1, 2, 4, 8, 16):
                    if name == "bf16":
                        f = lambda: ops.gemm_into(a, nxt(wb), out, force_cfg=1000 + kg)
                    else:
                        def f():
                            w, sc = nxt(w8)
                            torch.ops.shai.gemm(a, w, out, None, None, 1, None, 1.0, 1.0, 0, False, None, 1,
                                                1000 + kg, -1.0, sc)
                    try:
                        t = timeit(f, iters=48)
                    except Exception:  # noqa
                        continue
                    if name not in best or t < best[name][0]:
                        best[name] = (t, kg)
            del wb, w8
            gb = N * K * 2 / 1e9
            rows.append(dict(op="decode_fp8", shape=f"{M}x{N}x{K}", bf16_us=best["bf16"][0] * 1e6,
                             bf16_kg=best["bf16"][1], fp8_us=best["fp8"][0] * 1e6, fp8_kg=best["fp8"][1],
                             bf16_TBps=gb / best["bf16"][0] / 1e3, fp8_eqTBps=gb / best["fp8"][0] / 1e3))


def bench_sdgemm(rows):
    """SD2.1 batch-8 (CFG 16) transformer GEMMs: every tile config (forced) vs the tuned choice vs hipBLASLt."""
    shapes = [("sq4096", 4096, 4096, 4096, False), ("sq8192", 8192, 8192, 8192, False),
              ("geglu_L1", 65536, 2560, 320, True), ("ffdown_L1", 65536, 320, 1280, False),
              ("qkv_L1", 65536, 960, 320, False), ("proj_L1", 65536, 320, 320, False),
              ("geglu_L2", 16384, 5120, 640, True), ("ffdown_L2", 16384, 640, 2560, False),
              ("geglu_L3", 4096, 10240, 1280, True), ("ffdown_L3", 4096, 1280, 5120, False)]
    for name, M, N, K, glu in shapes:
        a, w = rnd(M, K), rnd(N, K) * (1 / math.sqrt(K))
        out = torch.empty(M, N // 2 if glu else N, device="cuda", dtype=torch.bfloat16)
        res = {}
        for c in range(7):
            res[c] = timeit(lambda: ops.gemm_into(a, w, out, act="gelu" if glu else None, glu=glu, force_cfg=c))
        t_tuned = timeit(lambda: ops.linear(a, w, act="gelu" if glu else None, glu=glu))
        t_t = timeit(lambda: torch.matmul(a, w.t()))
        f = 2 * M * N * K
        rows.append(dict(op=name, shape=f"{M}x{N}x{K}", **{f"cfg{c}_us": v * 1e6 for c, v in res.items()},
                         tuned_us=t_tuned * 1e6, torch_us=t_t * 1e6, tuned_tflops=f / t_tuned / 1e12,
                         torch_tflops=f / t_t / 1e12))


def bench_conv(rows):
    shapes = [(8, 64, 320, 320, 3), (8, 32, 640, 640, 3), (8, 16, 1280, 1280, 3), (8, 8, 1280, 1280, 3),
              (8, 64, 640, 320, 3), (1, 256, 256, 128, 3), (1, 512, 128, 128, 3), (8, 64, 320, 320, 1)]
    for N, H, C, Co, k in shapes:
        x = rnd(N, H, H, C)
        w4 = rnd(Co, C, k, k) * (1 / math.sqrt(C * k * k))
        wp = ops.pack_conv_weight(w4)
        b = rnd(Co)
        pad = k // 2
        t_s = timeit(lambda: ops.conv2d(x, wp, b, k, k, 1, pad))
        xc = x.permute(0, 3, 1, 2)  # channels_last view
        w4c = w4.contiguous(memory_format=torch.channels_last)
        t_t = timeit(lambda: F.conv2d(xc, w4c, b, padding=pad))
        f = 2 * N * H * H * Co * C * k * k
        rows.append(dict(op=f"conv{k}x{k}", shape=f"N{N} {H}x{H} {C}->{Co}", shai_us=t_s * 1e6, torch_us=t_t * 1e6,
                         shai_tflops=f / t_s / 1e12, torch_tflops=f / t_t / 1e12))


def bench_attn(rows):
    shapes = [(64, 4096, 4096, 5, 64), (8, 4096, 4096, 5, 64), (8, 1024, 1024, 10, 64), (8, 4096, 77, 5, 64),
              (1, 4608, 4608, 24, 128),
              (4, 2048, 2048, 32, 128), (16, 197, 197, 12, 64)]
    for B, Sq, Skv, H, D in shapes:
        q, k, v = rnd(B, Sq, H, D), rnd(B, Skv, H, D), rnd(B, Skv, H, D)
        t_s = timeit(lambda: ops.attention(q, k, v))
        qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        t_t = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt))
        f = 4 * B * H * Sq * Skv * D
        rows.append(dict(op="attn", shape=f"B{B} H{H} {Sq}x{Skv} d{D}", shai_us=t_s * 1e6, torch_us=t_t * 1e6,
                         shai_tflops=f / t_s / 1e12, torch_tflops=f / t_t / 1e12))


def bench_norm(rows):
    for N, HW, C in [(8, 4096, 320), (8, 1024, 640), (1, 262144, 128)]:
        x = rnd(N, HW, C)
        g, b = rnd(C), rnd(C)
        t_s = timeit(lambda: ops.groupnorm(x, g, b, 32, 1e-5, True))
        xt = x.view(N, HW, C).permute(0, 2, 1)
        t_t = timeit(lambda: F.silu(F.group_norm(xt, 32, g, b, 1e-5)))
        by = 3 * x.numel() * 2
        rows.append(dict(op="groupnorm+silu", shape=f"{N}x{HW}x{C}", shai_us=t_s * 1e6, torch_us=t_t * 1e6,
                         shai_GBps=by / t_s / 1e9, torch_GBps=by / t_t / 1e9))
    for T, D in [(8192, 4096), (64, 4096), (32768, 320)]:
        x, w = rnd(T, D), rnd(D)
        t_s = timeit(lambda: ops.rmsnorm(x, w, 1e-6))
        by = 2 * x.numel() * 2
        rows.append(dict(op="rmsnorm", shape=f"{T}x{D}", shai_us=t_s * 1e6, shai_GBps=by / t_s / 1e9))


def bench_f8(rows):
    """W8A8 fp8 MFMA GEMM (both tile configs, quantisation excluded / included) vs the bf16 GEMM on LLM prefill
    shapes; TF/s on the true FLOP count."""
    for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (4096, 28672, 4096), (4096, 4096, 14336),
                    (2048, 6144, 4096)]:
        x = rnd(M, K)
        w = rnd(N, K) / K ** 0.5
        a8, a_s = ops.quant_rows_fp8(x)
        w8, w_s = ops.quantize_fp8_rows(w)
        f = 2 * M * N * K
        t = {c: timeit(lambda: ops.gemm_f8(a8, w8, a_s, w_s, cfg=c)) for c in (0, 1, 2)}
        t_q = timeit(lambda: ops.linear(x, w8, w_scale=w_s))
        t_b = timeit(lambda: ops.linear(x, w))
        rows.append(dict(op="gemm_f8", shape=f"{M}x{N}x{K}", f8_256x128_us=t[0] * 1e6, f8_128x128_us=t[1] * 1e6,
                         f8_256x256_us=t[2] * 1e6,
                         f8_TFs=f / min(t.values()) / 1e12, w8a8_linear_TFs=f / t_q / 1e12,
                         bf16_TFs=f / t_b / 1e12))


def bench_dattn(rows):
    """Paged decode attention (Mistral-7B layer: 32 q heads, 8 KV heads, D 128), fused RoPE + KV write, per
    split count and context length; KV bytes read / time."""
    import math
    h, hk, D = 32, 8, 128
    shapes = [(64, 192), (64, 1024), (16, 4096), (1, 16384)]
    if os.environ.get("SHAI_DATTN_SHAPES"):  # e.g. "64x2,64x64,64x192": batch x context
        shapes = [tuple(int(v) for v in t.split("x")) for t in os.environ["SHAI_DATTN_SHAPES"].split(",")]
    for B, ctx in shapes:
        nblk = (ctx + 63) // 64
        pool = B * nblk + 8
        kc = rnd(pool, hk, 64, D)
        vc = rnd(pool, hk, 64, D)
        bt = torch.randperm(pool, device="cuda")[:B * nblk].view(B, nblk).int()
        ctx_l = torch.full((B,), ctx, device="cuda", dtype=torch.int32)
        pos = ctx_l - 1
        cos, sin = torch.rand(ctx + 1, D // 2, device="cuda"), torch.rand(ctx + 1, D // 2, device="cuda")
        slots = (bt[:, (ctx - 1) // 64] * 64 + (ctx - 1) % 64).int()
        qkv = rnd(B, (h + 2 * hk) * D)
        gb = B * hk * (ctx - 1) * D * 2 * 2 / 1e9
        r = dict(op="decode_attn", shape=f"B{B} ctx{ctx}")
        prev = ops.set_decode_wb(0)
        for sp in (1, 2, 4, 8, 16):
            if sp > nblk:
                continue
            t = timeit(lambda: ops.decode_attention_rope(qkv, kc, vc, bt, ctx_l, pos, cos, sin, slots, h, hk,
                                                         num_splits=sp), iters=48)
            r[f"s{sp}_us"] = t * 1e6
        ops.set_decode_wb(1)  # one split -> the wave-per-block kernel
        t = timeit(lambda: ops.decode_attention_rope(qkv, kc, vc, bt, ctx_l, pos, cos, sin, slots, h, hk,
                                                     num_splits=1), iters=48)
        r["wb_us"] = t * 1e6
        # graph-replayed (host launch cost out of the loop): split kernel vs wave-per-block, one split
        for mode, name in ((0, "g_s1_us"), (1, "g_wb_us")):
            ops.set_decode_wb(mode)
            o = torch.empty(B, h * D, device="cuda", dtype=torch.bfloat16)
            r[name] = graph_time(lambda: ops.decode_attention_rope(qkv, kc, vc, bt, ctx_l, pos, cos, sin, slots, h,
                                                                   hk, num_splits=1, out=o)) * 1e6
        ops.set_decode_wb(prev)
        best = min(v for k, v in r.items() if k.endswith("_us"))
        r["best_GBps"] = gb / (best / 1e6)
        r["auto_splits"] = ops.decode_splits(B, hk, ctx)
        rows.append(r)


def bench_dattn_long(rows):
    """Decode attention over one 128k-token context (plus 16 short sequences beside it), block tables contiguous
    vs scattered over a 4 GB-per-tensor pool, per split count: is the KV walk bound by page scatter (TLB) or by
    the per-workgroup block loop?"""
    h, hk, D = 32, 8, 128
    ctx = 131072
    nblk = ctx // 64
    pool = 32768
    kc = rnd(pool, hk, 64, D)
    vc = rnd(pool, hk, 64, D)
    cos, sin = torch.rand(ctx + 1, D // 2, device="cuda"), torch.rand(ctx + 1, D // 2, device="cuda")
    gb = hk * (ctx - 1) * D * 2 * 2 / 1e9
    for layout in ("contiguous", "scattered"):
        long_ids = (torch.arange(nblk, device="cuda") if layout == "contiguous"
                    else torch.randperm(pool, device="cuda")[:nblk])
        for B in (1, 17):
            bt = torch.zeros(B, nblk, dtype=torch.int32, device="cuda")
            bt[0] = long_ids.int()
            ctx_l = torch.full((B,), 256, device="cuda", dtype=torch.int32)
            ctx_l[0] = ctx
            for i in range(1, B):
                bt[i, :4] = torch.arange(pool - 4 * i, pool - 4 * i + 4, device="cuda").int()
            pos = ctx_l - 1
            slots = torch.stack([bt[i, (int(ctx_l[i]) - 1) // 64] * 64 + (int(ctx_l[i]) - 1) % 64
                                 for i in range(B)]).int()
            qkv = rnd(B, (h + 2 * hk) * D)
            r = dict(op="decode_attn_long", shape=f"B{B} ctx{ctx} {layout}")
            for sp in (16, 32, 64):
                t = timeit(lambda: ops.decode_attention_rope(qkv, kc, vc, bt, ctx_l, pos, cos, sin, slots, h, hk,
                                                             num_splits=sp), iters=20)
                r[f"s{sp}_us"] = t * 1e6
            best = min(v for k, v in r.items() if k.endswith("_us"))
            r["best_GBps"] = gb / (best / 1e6)
            rows.append(r)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gemm,conv,attn,norm")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    rows = []
    with torch.inference_mode():
        for name in a.only.split(","):
            {"gemm": bench_gemm, "conv": bench_conv, "attn": bench_attn, "norm": bench_norm,
             "decode": bench_decode, "decode_fp8": bench_decode_fp8, "sdgemm": bench_sdgemm, "f8": bench_f8,
             "dattn": bench_dattn, "dattn_long": bench_dattn_long}[name](rows)
    for r in rows:
        print("  ".join(f"{k}={v:.1f}" if isinstance(v, float) else f"{k}={v}" for k, v in r.items()), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
