"""Plain fp32 PyTorch reference of the Flux.1 transformer written directly from
diffusers' FluxTransformer2DModel semantics (diffusers itself is not installed in
this image, so parity against diffusers is unpinned; this reference pins the
fused/hoisted implementation against the textbook formulation with the SAME
diffusers-format state dict: separate q/k/v, explicit concat, unfused norms)."""
import math

import torch
import torch.nn.functional as F


def random_flux_state_dict(c, seed=0):
    g = torch.Generator().manual_seed(seed)
    d, D, mlp = c.hidden, c.head_dim, c.mlp_hidden

    def lin(name, i, o, sd):
        sd[name + ".weight"] = (torch.randn(o, i, generator=g) / math.sqrt(i)).to(torch.bfloat16)
        sd[name + ".bias"] = (torch.randn(o, generator=g) * 0.02).to(torch.bfloat16)

    sd = {}
    lin("x_embedder", c.in_channels, d, sd)
    lin("context_embedder", c.joint_attention_dim, d, sd)
    for e, din in (("timestep_embedder", 256), ("guidance_embedder", 256),
                   ("text_embedder", c.pooled_projection_dim)):
        if e == "guidance_embedder" and not c.guidance_embeds:
            continue
        lin(f"time_text_embed.{e}.linear_1", din, d, sd)
        lin(f"time_text_embed.{e}.linear_2", d, d, sd)
    for i in range(c.num_layers):
        p = f"transformer_blocks.{i}."
        lin(p + "norm1.linear", d, 6 * d, sd)
        lin(p + "norm1_context.linear", d, 6 * d, sd)
        for n in ("to_q", "to_k", "to_v", "add_q_proj", "add_k_proj", "add_v_proj", "to_add_out"):
            lin(p + "attn." + n, d, d, sd)
        lin(p + "attn.to_out.0", d, d, sd)
        for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k"):
            sd[p + f"attn.{n}.weight"] = (1 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16)
        for f in ("ff", "ff_context"):
            lin(p + f + ".net.0.proj", d, mlp, sd)
            lin(p + f + ".net.2", mlp, d, sd)
    for i in range(c.num_single_layers):
        p = f"single_transformer_blocks.{i}."
        lin(p + "norm.linear", d, 3 * d, sd)
        for n in ("to_q", "to_k", "to_v"):
            lin(p + "attn." + n, d, d, sd)
        for n in ("norm_q", "norm_k"):
            sd[p + f"attn.{n}.weight"] = (1 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16)
        lin(p + "proj_mlp", d, mlp, sd)
        lin(p + "proj_out", d + mlp, d, sd)
    lin("norm_out.linear", d, 2 * d, sd)
    lin("proj_out", d, c.in_channels, sd)
    return sd


def _lin(sd, name, x):
    return F.linear(x, sd[name + ".weight"].float(), sd[name + ".bias"].float())


def _tsin(t, dim=256):
    half = dim // 2
    ex = torch.exp(-math.log(10000) * torch.arange(half, dtype=torch.float32) / half)
    e = t.float()[:, None] * ex[None]
    return torch.cat([torch.cos(e), torch.sin(e)], -1)


def _rope(ids, axes, theta):
    cos, sin = [], []
    for i, d in enumerate(axes):
        freqs = 1.0 / (theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d))
        ang = ids[:, i:i + 1].double() * freqs[None]
        cos.append(torch.cos(ang).repeat_interleave(2, -1))
        sin.append(torch.sin(ang).repeat_interleave(2, -1))
    return torch.cat(cos, -1).float(), torch.cat(sin, -1).float()


def _apply_rope(x, cos, sin):  # x [B, H, S, D]
    xr, xi = x.reshape(*x.shape[:-1], -1, 2).unbind(-1)
    rot = torch.stack([-xi, xr], -1).flatten(3)
    return x * cos[None, None] + rot * sin[None, None]


def _rms(x, w, eps=1e-6):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def _ln(x, eps=1e-6):
    return F.layer_norm(x, (x.shape[-1],), eps=eps)


def flux_reference(sd, c, latents, t5, pooled, t, guidance, h2, w2):
    """Unfused fp32 forward. latents [B, Ni, 64], t5 [B, Nt, 4096], pooled [B, 768], t/guidance [B] in [0, 1]."""
    B, Ni, _ = latents.shape
    Nt = t5.shape[1]
    d, H, D = c.hidden, c.heads, c.head_dim
    img = _lin(sd, "x_embedder", latents.float())
    txt = _lin(sd, "context_embedder", t5.float())
    te = "time_text_embed."
    temb = _lin(sd, te + "timestep_embedder.linear_2", F.silu(_lin(sd, te + "timestep_embedder.linear_1",
                                                                   _tsin(t * 1000))))
    if c.guidance_embeds:
        temb = temb + _lin(sd, te + "guidance_embedder.linear_2",
                           F.silu(_lin(sd, te + "guidance_embedder.linear_1", _tsin(guidance * 1000))))
    temb = temb + _lin(sd, te + "text_embedder.linear_2", F.silu(_lin(sd, te + "text_embedder.linear_1",
                                                                       pooled.float())))
    ids = torch.zeros(Nt + Ni, 3)
    ids[Nt:, 1] = torch.arange(h2).repeat_interleave(w2).float()
    ids[Nt:, 2] = torch.arange(w2).repeat(h2).float()
    cos, sin = _rope(ids, c.axes_dims_rope, c.rope_theta)

    def heads(x):
        return x.view(B, -1, H, D).transpose(1, 2)

    for i in range(c.num_layers):
        p = f"transformer_blocks.{i}."
        m = _lin(sd, p + "norm1.linear", F.silu(temb)).chunk(6, -1)
        mc = _lin(sd, p + "norm1_context.linear", F.silu(temb)).chunk(6, -1)
        x = _ln(img) * (1 + m[1][:, None]) + m[0][:, None]
        cx = _ln(txt) * (1 + mc[1][:, None]) + mc[0][:, None]
        a = p + "attn."
        q = _rms(heads(_lin(sd, a + "to_q", x)), sd[a + "norm_q.weight"])
        k = _rms(heads(_lin(sd, a + "to_k", x)), sd[a + "norm_k.weight"])
        v = heads(_lin(sd, a + "to_v", x))
        cq = _rms(heads(_lin(sd, a + "add_q_proj", cx)), sd[a + "norm_added_q.weight"])
        ck = _rms(heads(_lin(sd, a + "add_k_proj", cx)), sd[a + "norm_added_k.weight"])
        cv = heads(_lin(sd, a + "add_v_proj", cx))
        q, k, v = torch.cat([cq, q], 2), torch.cat([ck, k], 2), torch.cat([cv, v], 2)
        q, k = _apply_rope(q, cos, sin), _apply_rope(k, cos, sin)
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, Nt + Ni, H * D)
        img = img + m[2][:, None] * _lin(sd, a + "to_out.0", o[:, Nt:])
        txt = txt + mc[2][:, None] * _lin(sd, a + "to_add_out", o[:, :Nt])
        x = _ln(img) * (1 + m[4][:, None]) + m[3][:, None]
        img = img + m[5][:, None] * _lin(sd, p + "ff.net.2", F.gelu(_lin(sd, p + "ff.net.0.proj", x), approximate="tanh"))
        cx = _ln(txt) * (1 + mc[4][:, None]) + mc[3][:, None]
        txt = txt + mc[5][:, None] * _lin(sd, p + "ff_context.net.2",
                                          F.gelu(_lin(sd, p + "ff_context.net.0.proj", cx), approximate="tanh"))
    h = torch.cat([txt, img], 1)
    for i in range(c.num_single_layers):
        p = f"single_transformer_blocks.{i}."
        sh, sc, gt = _lin(sd, p + "norm.linear", F.silu(temb)).chunk(3, -1)
        x = _ln(h) * (1 + sc[:, None]) + sh[:, None]
        mlp = F.gelu(_lin(sd, p + "proj_mlp", x), approximate="tanh")
        a = p + "attn."
        q = _apply_rope(_rms(heads(_lin(sd, a + "to_q", x)), sd[a + "norm_q.weight"]), cos, sin)
        k = _apply_rope(_rms(heads(_lin(sd, a + "to_k", x)), sd[a + "norm_k.weight"]), cos, sin)
        v = heads(_lin(sd, a + "to_v", x))
        o = F.scaled_dot_product_attention(q, k, v).transpose(1, 2).reshape(B, Nt + Ni, H * D)
        h = h + gt[:, None] * _lin(sd, p + "proj_out", torch.cat([o, mlp], -1))
    img = h[:, Nt:]
    sc, sh = _lin(sd, "norm_out.linear", F.silu(temb)).chunk(2, -1)
    img = _ln(img) * (1 + sc[:, None]) + sh[:, None]
    return _lin(sd, "proj_out", img)
