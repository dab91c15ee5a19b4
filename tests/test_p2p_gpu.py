"""Custom xGMI/IPC one-shot all-reduce (csrc/comm/p2p_allreduce.hip), two ranks sharing cuda:0."""
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def test_p2p_allreduce_two_ranks_one_gpu(cuda):
    import p2p_worker
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(p2p_worker.run, args=(2, port), nprocs=2, join=True)


def test_row_parallel_overlap_two_ranks_one_gpu(cuda):
    import tp_overlap_worker
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(tp_overlap_worker.run, args=(2, port), nprocs=2, join=True)
