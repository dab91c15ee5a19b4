#!/usr/bin/env python3
"""Per-shape device-time breakdown of one eager SD2.1 UNet step (random-init weights, batch B x 2 for CFG).

torch.profiler records every ``torch.ops.shai.*`` call with its input shapes; rows are grouped by
(op, shapes) and sorted by total device time.  Used to pick what to optimise next.

    python tools/op_breakdown.py [--batch 32] [--top 40]
"""
import argparse
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from shai_amd.models.unet2d import UNet2DConditionModel, UNetConfig  # noqa: E402
from shai_amd.weights import materialize  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    dev = "cuda:0"
    torch.manual_seed(0)
    unet = UNet2DConditionModel(UNetConfig.sd21())
    materialize(unet, dev)
    B = 2 * a.batch
    x = torch.randn(B, 64, 64, 4, device=dev).bfloat16()
    ctx = torch.randn(B, 77, 1024, device=dev).bfloat16()
    t = torch.tensor([500.0], device=dev)
    with torch.inference_mode():
        kv = unet.context_kv(ctx)
        for _ in range(2):
            unet(x, t, kv)
        torch.cuda.synchronize()
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA,
                                                torch.profiler.ProfilerActivity.CPU],
                                    record_shapes=True) as prof:
            unet(x, t, kv)
            torch.cuda.synchronize()
    rows = defaultdict(lambda: [0, 0.0])
    total = 0.0
    for ev in prof.key_averages(group_by_input_shape=True):
        dt = getattr(ev, "device_time_total", None)
        if dt is None:
            dt = ev.cuda_time_total
        if not ev.key.startswith("shai::") or dt <= 0:
            continue
        k = (ev.key, str(ev.input_shapes)[:150])
        rows[k][0] += ev.count
        rows[k][1] += dt
        total += dt
    print(f"total shai device time per UNet step (batch {B}): {total / 1e3:.2f} ms")
    print(f"{'ms':>8} {'%':>5} {'calls':>5} {'us/call':>8}  op  shapes")
    for (key, shp), (cnt, us) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{us / 1e3:8.3f} {100 * us / total:5.1f} {cnt:5d} {us / cnt:8.1f}  {key}  {shp}")


if __name__ == "__main__":
    main()
