"""One SD2.1 UNet 3x3 conv shape under PMC counters (argv: level = 320 / 640 / 1280, default 320): the batch-32 CFG
shape (64 images), NHWC, tuned kernel choice, 20 launches.  Run under
`rocprofv3 --pmc ... -- python3 tools/pmc_conv.py 320`."""
import sys

import torch

sys.path.insert(0, ".")
from shai_amd import ops  # noqa: E402


def main():
    lvl = int(sys.argv[1]) if len(sys.argv) > 1 else 320
    hw = {320: 64, 640: 32, 1280: 16}[lvl]
    x = torch.randn(64, hw, hw, lvl, device="cuda").bfloat16()
    w = ops.pack_conv_weight((torch.randn(lvl, lvl, 3, 3, device="cuda") / (9 * lvl) ** 0.5).bfloat16())
    b = torch.randn(lvl, device="cuda").bfloat16()
    for _ in range(20):
        ops.conv2d(x, w, b, 3, 3, 1, 1)
    torch.cuda.synchronize()
    print("done", lvl, flush=True)


if __name__ == "__main__":
    main()
