"""Decode GEMM under PMC counters: gate_up at M = 64 (64 x 28672 x 4096, rotating weight copies so every launch
streams HBM) with one forced kernel choice per run (argv[1] = force_cfg, e.g. 1201 skinny2, 1251 skinny2 6-stage,
1000 skinny v1).  Run under `rocprofv3 --pmc ... -- python3 tools/pmc_decode_gemm.py CFG`."""
import sys

import torch

sys.path.insert(0, ".")
import shai_amd  # noqa: E402,F401
from shai_amd import ops  # noqa: E402


def main():
    cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1201
    M, N, K = 64, 28672, 4096
    ncopy = 4
    a = torch.randn(M, K, device="cuda").bfloat16()
    ws = [(torch.randn(N, K, device="cuda") * 0.02).bfloat16() for _ in range(ncopy)]
    out = torch.empty(M, N // 2, device="cuda", dtype=torch.bfloat16)
    for i in range(64):
        ops.gemm_into(a, ws[i % ncopy], out, act="silu", glu=True, force_cfg=cfg, rms_eps=1e-5)
    torch.cuda.synchronize()
    print("done", cfg, flush=True)


if __name__ == "__main__":
    main()
