"""D = 128 attention: flash128x2 (two 32-query groups per wave, attention3.hip) vs flash2<128> (8-wave ping-pong,
attention2.hip) at the Flux joint-attention and LLM-prefill shapes, interleaved in one process (set_flash128x2)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from shai_amd import ops  # noqa: E402

SHAPES = [  # (B, S, H, Hkv, causal, label)
    (1, 4608, 24, 24, False, "Flux 1024^2 joint (24 x 128, 4608 tokens)"),
    (1, 1056, 24, 24, False, "Flux 512^2 joint (1056 tokens)"),
    (4, 2048, 32, 8, True, "Llama/Mistral prefill 4 x 2048, GQA 32/8, causal"),
    (1, 8192, 32, 8, True, "prefill 8192, GQA, causal"),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
    for i in range(n):
        ev[2 * i].record()
        fn()
        ev[2 * i + 1].record()
    torch.cuda.synchronize()
    return sorted(ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(n))[n // 2]


def main():
    K = ops._K()
    out = []
    for (B, S, H, Hk, causal, label) in SHAPES:
        torch.manual_seed(0)
        q = torch.randn(B, S, H, 128, device="cuda").bfloat16()
        k = torch.randn(B, S, Hk, 128, device="cuda").bfloat16()
        v = torch.randn(B, S, Hk, 128, device="cuda").bfloat16()
        res = {}
        for _ in range(2):
            for mode, name in ((1, "x2"), (0, "flash2")):
                K.set_flash128x2(mode)
                res.setdefault(name, []).append(timeit(lambda: ops.attention(q, k, v, causal=causal)))
        K.set_flash128x2(1)
        y1 = ops.attention(q, k, v, causal=causal)
        K.set_flash128x2(0)
        y0 = ops.attention(q, k, v, causal=causal)
        K.set_flash128x2(1)
        flop = 4.0 * B * H * S * S * 128 * (0.5 if causal else 1.0)
        row = {"shape": label}
        for n, ts in res.items():
            row[n + "_us"] = round(min(ts), 1)
            row[n + "_tfs"] = round(flop / min(ts) / 1e6, 1)
        row["max_abs_diff_vs_flash2"] = float((y1.float() - y0.float()).abs().max())
        out.append(row)
        print(json.dumps(row), flush=True)
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
