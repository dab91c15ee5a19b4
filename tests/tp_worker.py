"""Multi-process tensor-parallel checks (gloo on CPU): each rank builds the TP=world model from the
SAME full (unsharded) state dict via shard-on-load and compares against a TP=1 model in-process."""
import os

import torch


def _close(a, b, tol):
    a, b = a.float(), b.float()
    rel = ((a - b).norm() / (b.norm() + 1e-6)).item()
    assert rel < tol, f"rel err {rel}"


def _tp1():
    from shai_amd.parallel.state import TPState, set_tp
    set_tp(TPState())


def run(rank, world, port, which):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from shai_amd.models.layers import init_random_
    from shai_amd.parallel.state import init_distributed, set_tp
    from shai_amd.weights import load_into
    torch.manual_seed(0)
    if which == "llama":
        from shai_amd.engines.llm import LLMEngine, SamplingParams
        from shai_amd.models.llama import LlamaConfig, LlamaForCausalLM
        # 8 query heads / 2 KV heads: at TP 4 and 8 each rank holds a REPLICATED KV head (kv_heads < tp)
        c = LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                        num_attention_heads=8, num_key_value_heads=2, head_dim=32, max_position_embeddings=1024)
        _tp1()
        full = LlamaForCausalLM(c)
        init_random_(full, 3)
        sd = {k: v.clone() for k, v in full.state_dict().items()}
        n_dec = 10
        prompts = [[5, 9, 200, 31, 7], list(range(3, 80))]

        def run_engine(eng, forced=None):
            """Greedy generation recording the logits of every step (prefill, then n_dec - 1 decode steps).
            ``forced``: teacher forcing -- each step's appended tokens are replaced by the TP1 run's, so both
            runs see the same sequences even if an argmax flips under bf16 rounding."""
            rec = []
            fwd = eng.model.forward
            eng.model.forward = lambda *a, **k: (lambda y: (rec.append(y.float().clone()), y)[1])(fwd(*a, **k))
            p = SamplingParams(max_tokens=n_dec, temperature=0.0, ignore_eos=True)
            seqs = [eng.add_request(pr, p) for pr in prompts]
            row = {id(s): i for i, s in enumerate(seqs)}
            if forced is not None:
                app = eng._append
                eng._append = lambda ss, toks: app(ss, [forced[row[id(q)]][len(q.output)] for q in ss])
            while not all(q.finished for q in seqs):
                eng.step()
            return rec, [q.output for q in seqs]
        e1 = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False)
        load_into(e1.model, dict(sd), strict=True)
        ref_logits, ref_toks = run_engine(e1)
        assert len(ref_logits) == n_dec and all(len(t) == n_dec for t in ref_toks)
        init_distributed("gloo", tp_size=world)
        e2 = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False)
        assert e2.model.kv_heads_local == 1
        load_into(e2.model, dict(sd), strict=True)
        got_logits, got_toks = run_engine(e2, forced=ref_toks)
        assert got_toks == ref_toks
        assert len(got_logits) == len(ref_logits)
        for g, r in zip(got_logits, ref_logits):   # prefill logits, then every decode step's
            assert g.shape == r.shape
            _close(g, r, 3e-2)   # bf16 partial sums are rounded before the all-reduce at TP>1
        # random init is TP-consistent: a TP=world engine built from the seed alone equals the TP1 one
        st = init_distributed("gloo", tp_size=world)
        e3 = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False, seed=0)
        l3, _ = run_engine(e3)
        _tp1()
        e4 = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False, seed=0)
        l4, _ = run_engine(e4)
        set_tp(st)
        _close(l3[0], l4[0], 3e-2)
    elif which == "t5":
        from shai_amd.models.t5 import T5Config, T5EncoderModel
        c = T5Config(vocab_size=500, d_model=128, d_kv=16, d_ff=256, num_layers=2, num_heads=8)
        _tp1()
        m1 = T5EncoderModel(c)
        init_random_(m1, 4)
        sd = {k: v.clone() for k, v in m1.state_dict().items()}
        ids = torch.randint(2, 500, (2, 24))
        mask = torch.ones(2, 24, dtype=torch.long)
        mask[1, 15:] = 0
        ref = m1(ids, mask)
        init_distributed("gloo", tp_size=world)
        m2 = T5EncoderModel(c)
        load_into(m2, dict(sd), strict=True)
        _close(m2(ids, mask), ref, 3e-2)   # bf16 partial sums rounded before the all-reduce
    elif which in ("flux", "flux_sp", "flux_ovl"):
        # flux_sp: sequence-parallel single blocks (S/n-row residual shards, all-gather + reduce-scatter)
        # flux_ovl: every row-parallel GEMM chunked with its all-reduce overlapped
        if which == "flux_ovl":
            from shai_amd.parallel import comm
            comm.OVERLAP_MIN_ROWS, comm.OVERLAP_CHUNKS = 1, 2
        from shai_amd.models.flux import FluxConfig, FluxTransformer2DModel
        # 24 heads like Flux.1-dev: 3 heads per rank at TP 8 (app/src/transformer/model.py:163)
        c = FluxConfig(hidden=384, heads=24, head_dim=16, num_layers=2, num_single_layers=2,
                       joint_attention_dim=64, pooled_projection_dim=32, axes_dims_rope=(4, 6, 6))
        c.sequence_parallel = which == "flux_sp"
        B = 2 if c.sequence_parallel else 1
        _tp1()
        m1 = FluxTransformer2DModel(c)
        init_random_(m1, 5)
        sd = {k: v.clone() for k, v in m1.state_dict().items()}
        lat = torch.randn(B, 24, c.in_channels).bfloat16()
        t5 = torch.randn(B, 8, c.joint_attention_dim).bfloat16()
        pooled = torch.randn(B, c.pooled_projection_dim).bfloat16()
        t, g = torch.tensor([0.7] * B), torch.tensor([3.5] * B)
        with torch.no_grad():
            ref = m1(lat, t5, pooled, t, g, img_hw=(4, 6))
        init_distributed("gloo", tp_size=world)
        m2 = FluxTransformer2DModel(c)
        load_into(m2, dict(sd), strict=True)
        with torch.no_grad():
            _close(m2(lat, t5, pooled, t, g, img_hw=(4, 6)), ref, 3e-2)
    elif which == "mllama_vision":
        # the Llama-3.2-Vision tower head-sharded (QKV column-parallel by heads, o_proj / fc2 row-parallel, fc1
        # column-parallel) vs TP1, 3 valid tiles of 4 (padding queries take the exact masked path), gates folded
        from shai_amd.models.mllama import MllamaConfig, MllamaVisionModel
        vc = MllamaConfig.tiny().vision
        vc.attention_heads = 4
        _tp1()
        m1 = MllamaVisionModel(vc)
        init_random_(m1, 5)
        for lyr in m1.global_layers:   # non-trivial tanh gates
            lyr.gate_attn.fill_(0.7)
            lyr.gate_ffn.fill_(-0.4)
        sd = {k: v.clone() for k, v in m1.state_dict().items()}
        px = torch.randn(2, vc.max_num_tiles, vc.image_size, vc.image_size, 3).to(torch.bfloat16)
        ar = torch.tensor([3, 6])
        ref = m1(px, ar, [3, 4])
        init_distributed("gloo", tp_size=world)
        m2 = MllamaVisionModel(vc)
        assert m2.layers[0].self_attn.h == 4 // world
        load_into(m2, dict(sd), strict=True)
        _close(m2(px, ar, [3, 4]), ref, 3e-2)
    elif which == "row_overlap":
        # chunked row-parallel GEMM + all-reduce (compute / communication overlap path) vs the dense product
        from shai_amd.parallel import comm
        from shai_amd.parallel.layers import RowParallelLinear
        init_distributed("gloo", tp_size=world)
        comm.OVERLAP_MIN_ROWS, comm.OVERLAP_CHUNKS = 1, 3
        g = torch.Generator().manual_seed(5)
        w, b = torch.randn(48, 64, generator=g), torch.randn(48, generator=g)
        x, res = torch.randn(2, 300, 64, generator=g), torch.randn(2, 300, 48, generator=g)
        lin = RowParallelLinear(64, 48, bias=True, input_is_parallel=False, dtype=torch.float32)
        load_into(lin, {"weight": w, "bias": b}, strict=True)
        assert comm.overlap_chunks(600) == 3 and comm.overlap_chunks(2) == 2
        _close(lin(x, residual=res), x @ w.t() + b + res, 1e-5)
    elif which == "row_gated_slabs":
        # the slab schedule of the fused + overlapped row-parallel output stage (comm.row_parallel_reduce): 3 slabs
        # of 200 rows over 2 images of 300 rows, so a slab straddles the image boundary and the per-image AdaLN gate
        # is indexed from the slab's row offset; in place on the residual (the Flux gated update)
        from shai_amd.parallel import comm
        init_distributed("gloo", tp_size=world)
        assert comm.row_slabs(600, 3) == [(0, 200), (200, 400), (400, 600)]
        assert comm.row_slabs(601, 3) == [(0, 201), (201, 402), (402, 601)] and comm.row_slabs(2, 8) == [(0, 1), (1, 2)]
        g = torch.Generator().manual_seed(7)
        K, N = 64, 48
        w, b = torch.randn(N, K, generator=g), torch.randn(N, generator=g)
        x, res = torch.randn(2, 300, K, generator=g), torch.randn(2, 300, N, generator=g)
        mod = torch.randn(2, 3 * N, generator=g)
        gate = mod[:, N:2 * N]                      # strided column chunk of a modulation tensor
        want = res + gate[:, None, :] * (x @ w.t() + b)
        kl = K // world
        out = res.clone()
        y = comm.row_parallel_reduce(x[..., rank * kl:(rank + 1) * kl], w[:, rank * kl:(rank + 1) * kl], b, out,
                                     gate=gate, rows_per_gate=300, out=out, chunks=3)
        assert y is out
        _close(out, want, 1e-4)
    elif which == "seq_comm":
        from shai_amd.parallel import comm
        init_distributed("gloo", tp_size=world)
        full = [torch.randn(3, 4 * world, 5, generator=torch.Generator().manual_seed(r)) for r in range(world)]
        s = 4
        got = comm.all_gather_seq(full[rank][:, rank * s:(rank + 1) * s])
        want = torch.cat([full[r][:, r * s:(r + 1) * s] for r in range(world)], 1)
        assert torch.equal(got, want)
        rs = comm.reduce_scatter_seq(full[rank].clone())
        assert torch.allclose(rs, sum(full)[:, rank * s:(rank + 1) * s], atol=1e-5)
    elif which == "seq_gather_linears":
        # the SP all-gather forked beside the own rows' GEMMs (comm.gather_seq_linears): every rank's output equals
        # the dense GEMMs over the gathered sequence, at B = 1 and 2, into a strided column slice (the Flux single
        # blocks' [attn | mlp] buffer), and the GEMM schedule is own rows first, then the rows before / after
        from shai_amd import ops
        from shai_amd.parallel import comm
        init_distributed("gloo", tp_size=world)
        g = torch.Generator().manual_seed(11)
        d, s, N1, N2 = 32, 5, 24, 40
        w1, b1 = torch.randn(N1, d, generator=g), torch.randn(N1, generator=g)
        w2, b2 = torch.randn(N2, d, generator=g), torch.randn(N2, generator=g)
        for B in (1, 2):
            full = torch.randn(B, world * s, d, generator=g)
            out1 = torch.full((B, world * s, N1), float("nan"))
            cat = torch.full((B, world * s, 8 + N2), float("nan"))
            calls = []
            orig = ops.gemm_into

            def spy(x, w, out, *a, **k):
                calls.append(tuple(x.shape))
                return orig(x, w, out, *a, **k)
            ops.gemm_into = spy
            try:
                comm.gather_seq_linears(full[:, rank * s:(rank + 1) * s],
                                        [(w1, b1, None, out1), (w2, b2, "gelu_tanh", cat[..., 8:])])
            finally:
                ops.gemm_into = orig
            _close(out1, full @ w1.t() + b1, 1e-5)
            _close(cat[..., 8:], torch.nn.functional.gelu(full @ w2.t() + b2, approximate="tanh"), 1e-5)
            assert torch.isnan(cat[..., :8]).all()   # the columns left of the slice are untouched
            others = sum(j1 > j0 for j0, j1 in ((0, rank), (rank + 1, world)))
            assert calls[:2] == [(B, s, d)] * 2 and len(calls) == 2 * (1 + B * others), calls
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()
