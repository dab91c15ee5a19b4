"""VAE decoder A/B: whole-batch decode (operands > 2 GiB fall back to the v1 conv kernel) vs chunked decode.

python tools/bench_vae.py [--batch 32] [--res 512]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from shai_amd.models.layers import init_random_  # noqa: E402
from shai_amd.models.vae import AutoencoderKLDecoder, VAEConfig  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--res", type=int, default=512)
    a = ap.parse_args()
    with torch.device("cuda"):
        vae = init_random_(AutoencoderKLDecoder(VAEConfig.sd21()), seed=0).cuda()
    h = a.res // 8
    z = torch.randn(a.batch, h, h, 4, device="cuda").to(torch.bfloat16)
    default = vae.OPERAND_LIMIT
    with torch.inference_mode():
        for name, lim in (("whole", 1 << 62), ("chunked", default)):
            vae.OPERAND_LIMIT = lim
            for _ in range(2):
                vae(z)  # warm-up / GEMM autotune
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                vae(z)
            torch.cuda.synchronize()
            print(f"vae_decode mode={name} batch={a.batch} res={a.res} ms={(time.perf_counter() - t0) / 3 * 1e3:.1f}",
                  flush=True)


if __name__ == "__main__":
    main()
