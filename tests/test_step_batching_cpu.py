"""Step-level batching for SD2.1 (engines/diffusion.py StepBatcher): a request joining a running batch at a
step boundary, requests with different step counts, and the per-row fused scheduler update, all against the
one-request-at-a-time engine (tiny config, CPU)."""
import torch

from shai_amd.engines.diffusion import SDConfig, StableDiffusionEngine, StepBatcher


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-6)).item()


def test_step_batcher_matches_single_requests_with_mid_batch_join():
    eng = StableDiffusionEngine(SDConfig.tiny(), device="cpu")
    sb = StepBatcher(eng, max_batch=4)
    a = sb.add("a red fox", 6, seed=1)
    sb.step()
    sb.step()                                   # a is 2 steps in when b and c arrive
    b = sb.add("a blue hen", 4, seed=2)
    c = sb.add("a green owl", 5, seed=3)
    finished = []
    n_steps = 2
    while sb.has_work():
        finished += sb.step()
        n_steps += 1
    assert [r.done for r in (a, b, c)] == [True, True, True]
    assert n_steps == 7                         # 2 alone + max(4, 4, 5) with a finishing at step 6
    assert sb.stats["joined_mid_batch"] == 2
    for r, (p, s, seed) in ((a, ("a red fox", 6, 1)), (b, ("a blue hen", 4, 2)), (c, ("a green owl", 5, 3))):
        want = eng.generate([p], s, seed=seed)[0]
        assert r.image.shape == want.shape and r.image.dtype == torch.uint8
        assert (r.image.float() - want.float()).abs().mean() < 1.0, p


def test_step_batcher_capacity_and_order():
    eng = StableDiffusionEngine(SDConfig.tiny(), device="cpu")
    sb = StepBatcher(eng, max_batch=2)
    reqs = [sb.add(f"prompt {i}", 2, seed=i) for i in range(5)]
    order = []
    while sb.has_work():
        for r in sb.step():
            order.append(reqs.index(r))
        assert len(sb.active) <= 2
    assert sorted(order) == list(range(5)) and order[:2] == [0, 1]
    assert [StepBatcher.bucket(n) for n in (1, 3, 16, 17, 24, 25, 32)] == [1, 3, 16, 24, 24, 32, 32]
