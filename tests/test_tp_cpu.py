"""Tensor parallelism correctness by construction: TP=2 over gloo (two CPU processes, 127.0.0.1
rendezvous) reproduces TP=1 for the Llama engine (greedy tokens), the T5 encoder and the Flux MMDiT."""
import socket

import pytest
import torch.multiprocessing as mp

import tp_worker


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("which", ["llama", "t5", "flux", "flux_sp", "seq_comm"])
def test_tp2_matches_tp1(which):
    mp.spawn(tp_worker.run, args=(2, _port(), which), nprocs=2, join=True)


def test_seq_major_layout_is_rank_chunks():
    """The RCCL reduce-scatter input layout: chunk r of the rank-major view is sequence rows [r*s, (r+1)*s)."""
    import torch
    from shai_amd.parallel.comm import _seq_major
    for B in (1, 3):
        x = torch.randn(B, 12, 5)
        v = _seq_major(x, 4)
        assert v.is_contiguous() and v.shape == (4, B, 3, 5)
        for r in range(4):
            assert torch.equal(v[r], x[:, 3 * r:3 * (r + 1)])
