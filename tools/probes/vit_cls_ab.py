"""ViT-base b32 classification forward, HIP-graph replayed: the last layer for the CLS token only vs the full encoder.
    python tools/probes/vit_cls_ab.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from shai_amd.models.vit import ViTConfig, ViTForImageClassification  # noqa: E402


def main():
    torch.manual_seed(0)
    m = ViTForImageClassification(ViTConfig()).to("cuda").eval()
    for p in m.parameters():
        torch.nn.init.normal_(p, std=0.02)
    px = torch.randn(32, 224, 224, 3, device="cuda").bfloat16()
    res = {}
    with torch.inference_mode():
        for cls in (True, False):
            def fwd():
                h = m.vit(px, cls_only=cls)
                return m.classifier(h[:, 0].contiguous())
            for _ in range(3):
                out = fwd()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = fwd()
            g.replay()
            torch.cuda.synchronize()
            best = 1e30
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    g.replay()
                e1.record()
                e1.synchronize()
                best = min(best, e0.elapsed_time(e1) / 20)
            res[cls] = (best, out.float().clone())
    d = (res[True][1] - res[False][1]).abs().max().item()
    print(f"vit b32 forward: cls-only last layer {res[True][0] * 1000:.1f} us, full encoder {res[False][0] * 1000:.1f} us "
          f"({res[False][0] / res[True][0]:.3f}x); max |logit diff| {d:.4f}", flush=True)


if __name__ == "__main__":
    main()
