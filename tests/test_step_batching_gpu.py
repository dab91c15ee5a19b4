"""Step-level SD2.1 batching on the GPU (HIP-graph buckets with per-row timesteps + ops.sched_step_rows)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sched_step_rows_kernel(cuda):
    from shai_amd import ops
    from shai_amd.ops import reference as ref
    torch.manual_seed(0)
    B = 5
    lat = torch.randn(B, 16, 16, 4, device=cuda).bfloat16()
    mo = torch.randn(2 * B, 16, 16, 4, device=cuda).bfloat16()
    rows = torch.tensor([[0.5, 0.6, 0], [-1, 0, 0], [0.2, 0.3, 0], [0.9, 0.95, 0], [-1, 0, 0]], device=cuda)
    for pred in (0, 1):
        got = lat.clone()
        ops.sched_step_rows(mo, got, True, 7.5, pred, rows)
        want = lat.cpu().clone()
        ref.sched_step_rows(mo.cpu(), want, True, 7.5, pred, rows.cpu())
        assert torch.allclose(got.cpu().float(), want.float(), atol=2e-2, rtol=2e-2)
        assert torch.equal(got[1], lat[1]) and torch.equal(got[4], lat[4])


def test_step_batcher_gpu_matches_generate(cuda):
    from shai_amd.engines.diffusion import SDConfig, StableDiffusionEngine, StepBatcher
    eng = StableDiffusionEngine(SDConfig.tiny(), device="cuda")
    sb = StepBatcher(eng, max_batch=4)
    assert sb.warmup() == 4
    a = sb.add("a red fox", 6, seed=1)
    with torch.inference_mode():
        sb.step()
        b = sb.add("a blue hen", 4, seed=2)
        while sb.has_work():
            sb.step()
        for r, p, n, s in ((a, "a red fox", 6, 1), (b, "a blue hen", 4, 2)):
            want = eng.generate([p], n, seed=s)[0]
            # the batched bucket runs other GEMM configurations (per-shape autotune; the device debug build's
            # timings pick others again), so bf16 rounding differs: uint8 pixels agree to a level or two
            d = (r.image.float() - want.float()).abs()
            assert d.mean() < 2.0 and (d <= 2).float().mean() > 0.9, (d.mean(), (d <= 2).float().mean())
    assert sb.stats["joined_mid_batch"] == 1
