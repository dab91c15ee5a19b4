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


@pytest.mark.parametrize("which", ["llama", "t5", "flux", "flux_sp", "flux_ovl", "row_overlap", "row_gated_slabs",
                                   "seq_comm", "seq_gather_linears", "mllama_vision"])
def test_tp2_matches_tp1(which):
    mp.spawn(tp_worker.run, args=(2, _port(), which), nprocs=2, join=True)


@pytest.mark.slow
@pytest.mark.parametrize("world", [4, 8])
@pytest.mark.parametrize("which", ["llama", "t5", "flux", "flux_sp"])
def test_tp_degrees_4_8_match_tp1(which, world):
    """The TP degrees the reference runs (TP8: app/src/transformer/compile.py:25,
    app/src/text_encoder_2/compile.py:24): Llama with kv_heads < tp (replicated KV heads) checked on prefill
    AND 10 teacher-forced decode steps, T5 with 1 head per rank at TP8, Flux with 24 heads (3 per rank at
    TP8) with and without sequence parallelism."""
    mp.spawn(tp_worker.run, args=(world, _port(), which), nprocs=world, join=True)


def test_sp_gather_linears_middle_ranks():
    """World 4: ranks 1 and 2 have rows both before and after their own (two batched GEMMs per image after the
    join), ranks 0 / 3 only one side."""
    mp.spawn(tp_worker.run, args=(4, _port(), "seq_gather_linears"), nprocs=4, join=True)


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


def test_reduce_scatter_semantics_on_seq_major_b_gt_1():
    """Emulates RCCL reduce_scatter_tensor on the rank-major input (output r = sum over ranks of flat chunk r)
    for B > 1 and checks it equals the all-reduce result sliced to rank r's sequence rows."""
    import torch
    from shai_amd.parallel.comm import _seq_major
    n, B, S, d = 4, 3, 16, 6
    parts = [torch.randn(B, S, d, dtype=torch.float64) for _ in range(n)]
    full = sum(parts)
    flats = [_seq_major(p, n).reshape(n, -1) for p in parts]        # what the collective sees: n flat chunks
    s = S // n
    for r in range(n):
        out = sum(f[r] for f in flats).view(B, s, d)
        assert torch.allclose(out, full[:, r * s:(r + 1) * s])


def _rs_no_alias_worker(rank, world, port):
    import os
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from shai_amd.parallel.comm import reduce_scatter_seq
    g = dist.new_group(list(range(world)))
    x = torch.full((2, 4, 3), float(rank + 1))
    keep = x.clone()
    y = reduce_scatter_seq(x, group=g)
    assert torch.equal(x, keep), "reduce_scatter_seq modified its input"
    assert torch.allclose(y, torch.full((2, 2, 3), 3.0))
    dist.destroy_process_group()


def test_reduce_scatter_seq_gloo_keeps_input():
    mp.spawn(_rs_no_alias_worker, args=(2, _port()), nprocs=2, join=True)


def test_overlap_chunks_default_by_rows_and_bytes(monkeypatch):
    """The default row-slab count of the overlapped row-parallel stage is a function of rows and message size
    (comm.overlap_chunks): 4 slabs from 4096 rows (Flux 1024^2 TP8: 4608 rows, <= 1/4 of the 27 MiB reduce
    exposed), 2 from 1024 rows (Flux 512^2: 1056), none below 1024 rows or under 2 MiB; the env/attribute pin
    overrides it."""
    import types
    from shai_amd.parallel import comm
    monkeypatch.setattr(comm, "tp", lambda: types.SimpleNamespace(size=8, rank=0, group=None))
    monkeypatch.setattr(comm, "OVERLAP_CHUNKS", None)
    monkeypatch.setattr(comm, "OVERLAP_MIN_ROWS", 1024)
    assert comm.overlap_chunks(4608, 3072) == 4          # Flux 1024^2 single / dual image stream
    assert comm.overlap_chunks(4096, 3072) == 4
    assert comm.overlap_chunks(1056, 3072) == 2          # Flux 512^2
    assert comm.overlap_chunks(1023, 3072) == 1
    assert comm.overlap_chunks(2048, 256) == 1           # 1 MiB: latency-bound, no split
    assert comm.overlap_chunks(2048) == 2                # width unknown: rows decide
    assert [b - a for a, b in comm.row_slabs(4608, 4)] == [1152] * 4
    monkeypatch.setattr(comm, "OVERLAP_CHUNKS", 3)
    assert comm.overlap_chunks(4608, 3072) == 3 and comm.overlap_chunks(512, 3072) == 1
    monkeypatch.setattr(comm, "tp", lambda: types.SimpleNamespace(size=1, rank=0, group=None))
    assert comm.overlap_chunks(4608, 3072) == 1
