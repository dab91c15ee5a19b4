"""Process-group state: one process per GPU, ``torch.distributed`` over RCCL
(backend "nccl" on ROCm) on GPUs, gloo on CPU (tests).

The reference has no explicit collectives: its TP lives inside NxD
``parallel_state`` / NEFFs (app/src/transformer/model.py:7-9,143-159).  Here a
tensor-parallel group is an explicit ``ProcessGroup`` and collectives are issued
by the TP layers (``shai_amd.parallel.layers``) through ``shai_amd.parallel.comm``.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class TPState:
    rank: int = 0
    size: int = 1
    group: Optional[dist.ProcessGroup] = None
    device: torch.device = torch.device("cpu")


_TP = TPState()


def init_distributed(backend: Optional[str] = None, tp_size: Optional[int] = None,
                     device: Optional[str] = None) -> TPState:
    """Initialise the default process group from torchrun env vars and make the
    (single) tensor-parallel group span ``tp_size`` consecutive ranks.

    GPUs: backend "nccl" (RCCL) with one GPU per rank; every TP group of size > 1 also gets the xGMI P2P
    all-reduce / all-gather (``SHAI_P2P_ALLREDUCE=0`` disables it).  ``device="cuda"`` with backend "gloo" puts
    every rank on GPU ``LOCAL_RANK % device_count`` with gloo only for host-side coordination -- several ranks
    sharing ONE GPU (tests): then the model's collectives must fit the P2P kernels."""
    global _TP
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and (backend != "gloo" or device == "cuda")
    if use_gpu:
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        be = backend or ("nccl" if use_gpu else "gloo")
        if be == "nccl":
            dist.init_process_group(be, device_id=device)
        else:
            dist.init_process_group(be)
    tp = tp_size or world
    assert world % tp == 0, f"world {world} not divisible by tp {tp}"
    group = None
    if world > 1 and tp > 1:
        for start in range(0, world, tp):
            ranks = list(range(start, start + tp))
            g = dist.new_group(ranks)
            if rank in ranks:
                group = g
    _TP = TPState(rank % tp if tp > 1 else 0, tp, group, device)
    if tp > 1 and use_gpu and os.environ.get("SHAI_P2P_ALLREDUCE", "1") != "0":
        # custom xGMI peer all-reduce / all-gather for the TP group (small, latency-bound messages); RCCL for
        # the rest
        from .comm import P2PAllReduce, enable_p2p, p2p
        if p2p() is None or p2p().world != tp:
            enable_p2p(P2PAllReduce(group))
    return _TP


def set_tp(state: TPState) -> None:
    global _TP
    _TP = state


def tp() -> TPState:
    return _TP


def tp_rank() -> int:
    return _TP.rank


def tp_size() -> int:
    return _TP.size
