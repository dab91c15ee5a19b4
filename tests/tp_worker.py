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
        c = LlamaConfig.tiny()
        _tp1()
        full = LlamaForCausalLM(c)
        init_random_(full, 3)
        sd = {k: v.clone() for k, v in full.state_dict().items()}
        e1 = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False)
        load_into(e1.model, dict(sd), strict=True)
        p = SamplingParams(max_tokens=1, temperature=0.0, ignore_eos=True)
        prompts = [[5, 9, 200, 31, 7], list(range(3, 80))]

        def prefill_logits(eng):
            rec = []
            orig = eng._sample_and_append
            eng._sample_and_append = lambda seqs, logits: (rec.append(logits.float().clone()), orig(seqs, logits))
            eng.generate(prompts, p)
            return rec[0]
        ref = prefill_logits(e1)
        init_distributed("gloo", tp_size=world)
        e2 = LLMEngine(c, device="cpu", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False)
        load_into(e2.model, dict(sd), strict=True)
        got = prefill_logits(e2)
        assert got.shape == ref.shape
        _close(got, ref, 3e-2)   # bf16 partial sums are rounded before the all-reduce at TP>1
    elif which == "t5":
        from shai_amd.models.t5 import T5Config, T5EncoderModel
        c = T5Config.tiny()
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
        _close(m2(ids, mask), ref, 1e-2)
    elif which in ("flux", "flux_sp", "flux_ovl"):
        # flux_sp: sequence-parallel single blocks (S/n-row residual shards, all-gather + reduce-scatter)
        # flux_ovl: every row-parallel GEMM chunked with its all-reduce overlapped
        if which == "flux_ovl":
            from shai_amd.parallel import comm
            comm.OVERLAP_MIN_ROWS, comm.OVERLAP_CHUNKS = 1, 2
        from shai_amd.models.flux import FluxConfig, FluxTransformer2DModel
        c = FluxConfig.tiny()
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
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()
