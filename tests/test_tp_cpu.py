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


@pytest.mark.parametrize("which", ["llama", "t5", "flux"])
def test_tp2_matches_tp1(which):
    mp.spawn(tp_worker.run, args=(2, _port(), which), nprocs=2, join=True)
