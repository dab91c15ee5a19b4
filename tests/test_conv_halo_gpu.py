"""Halo-tiled 3x3 conv with the GroupNorm + SiLU prologue in LDS (csrc/kernels/conv_halo.hip) vs the fp32 PyTorch
reference of the same op (normalise -> SiLU -> zero-padded conv -> bias + time embedding + residual), at the SD2.1
UNet / VAE geometries: every supported row width (64 / 32 / 16 pixels: 4 / 8 / 16 rows per tile), both N tiles
(160 / 128 columns), the two-source channel concat of the up blocks, both wave layouts (4 and 8 waves), the
nearest-2x upsample variant (plain input), and the GroupNorm column partials its epilogue hands to the next norm.
Shapes it does not take (8 x 8 images, N = 4) run the apply-pass fallback inside the same op and are checked too."""
import pytest
import torch

from shai_amd import ops
from shai_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def _case(cuda, N, H, W, C1, C2, Cout, seed, temb=True, res=True, gn_dc=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.randn(N, H, W, C1, generator=g) * 1.5 + gn_dc).bfloat16().to(cuda)
    x2 = (torch.randn(N, H, W, C2, generator=g) - 0.5).bfloat16().to(cuda) if C2 else None
    cin = C1 + C2
    w = (torch.randn(Cout, 9 * cin, generator=g) / (9 * cin) ** 0.5).bfloat16().to(cuda)
    b = (0.1 * torch.randn(Cout, generator=g)).bfloat16().to(cuda)
    t = (0.1 * torch.randn(N, Cout, generator=g)).bfloat16().to(cuda) if temb else None
    r = torch.randn(N, H, W, Cout, generator=g).bfloat16().to(cuda) if res else None
    gamma = (1 + 0.2 * torch.randn(cin, generator=g)).bfloat16().to(cuda)
    beta = (0.2 * torch.randn(cin, generator=g)).bfloat16().to(cuda)
    sc, sh = ops.groupnorm_stats(x, gamma, beta, 32, 1e-5, x2=x2)
    return x, x2, w, b, t, r, sc, sh


def _want(x, x2, w, b, t, r, sc, sh, upsample=False, norm=True):
    cpu = lambda v: v.cpu() if v is not None else None  # noqa: E731
    return ref.conv2d(cpu(x), cpu(w), cpu(b), 3, 3, 1, 1, upsample, cpu(x2),
                      (cpu(sc), cpu(sh), "silu") if norm else None, cpu(t), cpu(r))


@pytest.fixture(autouse=True)
def _restore_mode():
    prev = ops.set_halo_conv(-1, -1)
    yield
    ops.set_halo_conv(prev, 0)


def test_default_mode_is_apply_pass(cuda):
    """Off by default (profiles/halo_conv_round6.md): norm= convs take the apply pass + tuned conv."""
    assert ops.set_halo_conv(-1, -1) == 0


@pytest.mark.parametrize("waves", [8, 4])
@pytest.mark.parametrize("N,H,W,C1,C2,Cout", [
    (2, 64, 64, 320, 0, 320),     # UNet 64x64 level: 4 rows per tile, two 160-column N tiles
    (2, 64, 64, 320, 320, 320),   # up-block concat (x 320 | skip 320)
    (2, 32, 32, 640, 320, 640),   # 32x32 level: 8 rows per tile, concat 640 | 320
    (1, 16, 16, 1280, 0, 1280),   # 16x16: one image per tile, 8 N tiles
    (1, 64, 64, 512, 0, 512),     # VAE 64x64 level: 128-column N tiles
])
def test_halo_gn_conv_matches_fp32(cuda, waves, N, H, W, C1, C2, Cout):
    ops.set_halo_conv(1, waves)
    x, x2, w, b, t, r, sc, sh = _case(cuda, N, H, W, C1, C2, Cout, seed=N * H + C1 + C2 + Cout, gn_dc=3.0)
    y, part = ops.conv2d(x, w, b, 3, 3, 1, 1, x2=x2, norm=(sc, sh, "silu"), temb=t, residual=r, stats="gn")
    want = _want(x, x2, w, b, t, r, sc, sh)
    assert _rel(y, want) < 1e-2
    # column partials of the stored output (the next GroupNorm's statistics) vs a pass over y
    assert part is not None
    pref = ref.col_partials(y.reshape(-1, Cout).cpu())
    assert _rel(part, pref) < 1e-4


def test_halo_matches_apply_pass_path(cuda):
    """The fused kernel and the fallback (apply pass + tuned conv, halo off) agree to bf16 rounding."""
    x, x2, w, b, t, r, sc, sh = _case(cuda, 2, 32, 32, 640, 0, 640, seed=5)
    ops.set_halo_conv(1, 0)
    y1 = ops.conv2d(x, w, b, 3, 3, 1, 1, norm=(sc, sh, "silu"), temb=t, residual=r)
    ops.set_halo_conv(0, 0)
    y0 = ops.conv2d(x, w, b, 3, 3, 1, 1, norm=(sc, sh, "silu"), temb=t, residual=r)
    assert _rel(y1, y0) < 5e-3


@pytest.mark.parametrize("H,Cout", [(8, 1280), (64, 4)])
def test_unsupported_shapes_take_the_apply_fallback(cuda, H, Cout):
    """8 x 8 images (64-pixel images: no 256-pixel tile) and N = 4 (UNet conv_out) run apply pass + conv."""
    Cin = 1280 if H == 8 else 320
    x, x2, w, b, t, r, sc, sh = _case(cuda, 2, H, H, Cin, 0, Cout, seed=H, temb=False, res=False)
    y = ops.conv2d(x, w, b, 3, 3, 1, 1, norm=(sc, sh, "silu"))
    assert _rel(y, _want(x, None, w, b, None, None, sc, sh)) < 1e-2


@pytest.mark.parametrize("waves", [8, 4])
def test_halo_plain_and_upsample(cuda, waves):
    """Mode 2: plain 3x3 convs (no norm) and the nearest-2x upsample conv of the up blocks on the halo kernel."""
    ops.set_halo_conv(2, waves)
    x, _, w, b, _, r, sc, sh = _case(cuda, 2, 32, 32, 640, 0, 640, seed=9, temb=False)
    y = ops.conv2d(x, w, b, 3, 3, 1, 1, upsample=True)
    assert _rel(y, _want(x, None, w, b, None, None, sc, sh, upsample=True, norm=False)) < 1e-2
    y = ops.conv2d(x, w, b, 3, 3, 1, 1, residual=r)
    assert _rel(y, _want(x, None, w, b, None, r, sc, sh, norm=False)) < 1e-2


def test_padding_is_zero_after_the_norm(cuda):
    """A large shift makes silu(shift) far from 0: the halo's padding pixels must stay exactly zero AFTER the norm
    (a kernel that normalised the zero fill would shift every border output)."""
    ops.set_halo_conv(1, 0)
    x, _, w, b, _, _, sc, sh = _case(cuda, 1, 16, 16, 640, 0, 640, seed=3, temb=False, res=False)
    assert ops.set_halo_conv(-1, -1) == 1
    sh = sh + 4.0
    ss = torch.stack([sc, sh]).contiguous()   # one allocation, as the kernel reads it
    y = ops.conv2d(x, w, b, 3, 3, 1, 1, norm=(ss[0], ss[1], "silu"))
    want = _want(x, None, w, b, None, None, ss[0], ss[1])
    assert _rel(y, want) < 1e-2
    assert _rel(y[:, 0], want[:, 0]) < 1e-2 and _rel(y[:, :, -1], want[:, :, -1]) < 1e-2
