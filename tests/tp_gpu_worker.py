"""Two ranks sharing ONE GPU run a TP=2 LLM engine (gloo only for host coordination; every collective of
the model -- the row-parallel all-reduces, the vocab-parallel embedding all-reduce, the logits all-gather --
goes through the xGMI/IPC P2P kernels, which init_distributed enables by default for TP > 1).  Checked
against a TP=1 engine built from the same seed on the same GPU: prefill + 8 teacher-forced decode steps
(logits), and the async look-ahead engine (HIP graphs) reproducing the sync engine's tokens exactly."""
import os

import torch


def _close(a, b, tol):
    rel = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-6)).item()
    assert rel < tol, f"rel err {rel}"


def run(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHAI_P2P_MAX_BLOCKS="128", SHAI_P2P_TIMEOUT_S="10")
    import torch.distributed as dist
    from shai_amd.engines.llm import LLMEngine, SamplingParams
    from shai_amd.models.llama import LlamaConfig
    from shai_amd.parallel import comm
    from shai_amd.parallel.state import TPState, init_distributed, set_tp
    torch.cuda.set_device(0)
    c = LlamaConfig(vocab_size=1024, hidden_size=512, intermediate_size=1024, num_hidden_layers=2,
                    num_attention_heads=8, num_key_value_heads=2, head_dim=64, max_position_embeddings=1024)
    prompts = [[5, 9, 200, 31, 7], list(range(3, 100))]
    n_dec = 9

    def run_engine(eng, forced=None):
        rec = []
        fwd = eng.model.forward
        eng.model.forward = lambda *a, **k: (lambda y: (rec.append(y.float().clone()), y)[1])(fwd(*a, **k))
        p = SamplingParams(max_tokens=n_dec, temperature=0.0, ignore_eos=True)
        seqs = [eng.add_request(pr, p) for pr in prompts]
        row = {id(s): i for i, s in enumerate(seqs)}
        app = eng._append
        if forced is not None:
            eng._append = lambda ss, toks: app(ss, [forced[row[id(q)]][len(q.output)] for q in ss])
        while not all(q.finished for q in seqs):
            eng.step()
        while eng.has_work():   # retire a look-ahead step past the last token
            eng.step()
        eng.model.forward = fwd
        eng._append = app
        return rec, [q.output for q in seqs]

    with torch.inference_mode():
        set_tp(TPState(device=torch.device("cuda", 0)))
        e1 = LLMEngine(c, device="cuda:0", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False, seed=0, use_graphs=False)
        ref_logits, ref_toks = run_engine(e1)
        del e1
        init_distributed("gloo", tp_size=world, device="cuda")
        assert comm.p2p() is not None, "P2P collectives must be on by default at TP > 1"
        # teacher-forced logits, sync engine, eager (the recorded forwards are the real ones)
        e2 = LLMEngine(c, device="cuda:0", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False, seed=0, use_graphs=False)
        got_logits, got_toks = run_engine(e2, forced=ref_toks)
        assert got_toks == ref_toks
        assert len(got_logits) == len(ref_logits) == n_dec, (len(got_logits), len(ref_logits))
        for g, r in zip(got_logits, ref_logits):
            assert g.shape == r.shape
            _close(g, r, 3e-2)
        _, eager_toks = run_engine(e2)                    # free-running (TP2 numerics)
        # HIP graphs (the decode graph captures the P2P all-reduces / all-gather), sync and async look-ahead:
        # the same tokens bit for bit
        e3 = LLMEngine(c, device="cuda:0", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=False, seed=0)
        _, sync_toks = run_engine(e3)
        e4 = LLMEngine(c, device="cuda:0", max_num_seqs=2, max_model_len=256, enable_prefix_caching=False,
                       async_decode=True, seed=0)
        _, async_toks = run_engine(e4)
        assert sync_toks == eager_toks, (sync_toks, eager_toks)
        assert async_toks == sync_toks, (async_toks, sync_toks)
        torch.cuda.synchronize()
        assert not comm.p2p().error()
    dist.barrier()
    comm.p2p().close()
    comm.enable_p2p(None)
    dist.destroy_process_group()


def run_flux(rank, world, port):
    """Flux pipeline (CLIP + T5 + MMDiT + VAE) at TP=2 on one GPU with HIP-graph steps vs TP=1 from the same
    seeds: every row-parallel all-reduce inside the captured step goes through the P2P kernels."""
    # one-shot only below 4 KiB: the tiny model's row-parallel messages then take the two-shot kernel through
    # the default routing (the path Flux's 6-27 MiB TP8 messages take)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SHAI_P2P_MAX_BLOCKS="128", SHAI_P2P_TIMEOUT_S="10",
                      SHAI_P2P_ONE_SHOT_MAX=str(4096))
    import torch.distributed as dist
    from shai_amd.engines.flux import FluxEngine, FluxPipelineConfig
    from shai_amd.parallel import comm
    from shai_amd.parallel.state import TPState, init_distributed, set_tp
    from shai_amd.models.flux import FluxConfig
    torch.cuda.set_device(0)
    comm.P2P_ONE_SHOT_MAX = 4096

    def cfg():  # head dims the GPU flash kernel takes (64 / 128), heads divisible by the TP degree
        c = FluxPipelineConfig.tiny()
        c.transformer = FluxConfig(hidden=256, heads=2, head_dim=128, num_layers=2, num_single_layers=2,
                                   joint_attention_dim=128, pooled_projection_dim=128, axes_dims_rope=(16, 56, 56))
        c.clip.hidden_size, c.clip.num_attention_heads, c.clip.intermediate_size = 128, 2, 256
        c.t5.d_model = 128
        return c
    with torch.inference_mode():
        set_tp(TPState(device=torch.device("cuda", 0)))
        e1 = FluxEngine(cfg(), device="cuda:0")
        ref = e1.generate(["a cat holding a sign"], 3, seed=5, output="tensor").float()
        other = e1.generate(["a cat holding a sign"], 3, seed=6, output="tensor").float()
        del e1
        init_distributed("gloo", tp_size=world, device="cuda")
        assert comm.p2p() is not None
        e2 = FluxEngine(cfg(), device="cuda:0")
        for _ in range(2):   # first call captures the step graph, second replays it
            got = e2.generate(["a cat holding a sign"], 3, seed=5, output="tensor").float()
            rel = ((got - ref).norm() / ref.norm()).item()
            rel_seed = ((other - ref).norm() / ref.norm()).item()
            assert rel < 5e-2 and rel < 0.1 * rel_seed, (rel, rel_seed)
        torch.cuda.synchronize()
        assert not comm.p2p().error()
        n = comm.p2p().launch_counts()
        # the gated row-parallel outputs ran as GEMM-into-the-slot + the fused two-shot reduce
        assert n["staged_two_shot"] > 0, n
    dist.barrier()
    comm.p2p().close()
    comm.enable_p2p(None)
    dist.destroy_process_group()
