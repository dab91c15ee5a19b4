"""Checkpoint loading: safetensors from a local directory (streamed, never
pickle), HF/diffusers key conversion per model, per-rank shard-on-load for
tensor parallel layers (TP layers slice rows/cols in their
``_load_from_state_dict`` hooks, so no pre-sharded files are needed), or
deterministic random init when no checkpoint is available (the offline GPU
box).  Replaces the reference's HF-Hub snapshot / ``parallel_model_load``
artifact flow (app/download_hf_model.py:1-8, app/t5_model_api.py:27-33).

Pre-sharded restart cache: with ``SHAI_SHARD_CACHE=<dir>`` (or
``materialize(shard_cache=...)``) the first load of a checkpoint writes this rank's
already-sliced, already-converted tensors to ``<dir>/tp{rank}of{size}.safetensors``; a
restarted worker loads only its own shard from there (no full-checkpoint read, no key
conversion, no slicing) -- the counterpart of the reference's per-rank ``tp_*.pt``
artifacts (app/t5_model_api.py:27, app/flux_model_api.py:130-140), produced on the fly
instead of by an offline compile job.  The file's metadata pins the model class and TP
layout; a mismatching or unreadable file is ignored and rebuilt.
"""
from __future__ import annotations

import glob
import os
from typing import Callable, Dict, Optional

import torch
import torch.nn as nn

from ..models.layers import init_random_


def find_safetensors(path: str, subfolder: Optional[str] = None):
    d = os.path.join(path, subfolder) if subfolder else path
    if os.path.isfile(d) and d.endswith(".safetensors"):
        return [d]
    return sorted(glob.glob(os.path.join(d, "*.safetensors")))


def load_safetensors(files) -> Dict[str, torch.Tensor]:
    from safetensors import safe_open
    sd = {}
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as h:
            for k in h.keys():
                sd[k] = h.get_tensor(k)
    return sd


def load_into(model: nn.Module, sd: Dict[str, torch.Tensor], convert: Optional[Callable] = None,
              strict: bool = False) -> nn.Module:
    if convert is not None:
        sd = convert(sd)
    dtype = next(model.parameters()).dtype
    sd = {k: (v.to(dtype) if v.is_floating_point() else v) for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    if strict and (missing or unexpected):
        raise RuntimeError(f"checkpoint mismatch: missing={missing[:10]} unexpected={unexpected[:10]}")
    return model


def _tp_layout():
    from ..parallel.state import tp
    st = tp()
    return st.rank, st.size


def shard_cache_path(cache_dir: str, rank: int, size: int) -> str:
    return os.path.join(cache_dir, f"tp{rank}of{size}.safetensors")


def _layout_meta(model: nn.Module, size: int) -> Dict[str, str]:
    sd = model.state_dict()
    sig = ";".join(f"{k}:{tuple(v.shape)}" for k, v in sorted(sd.items()))
    import hashlib
    return {"shai_class": type(model).__name__, "tp_size": str(size),
            "layout": hashlib.sha1(sig.encode()).hexdigest()}


def save_shard(model: nn.Module, cache_dir: str) -> str:
    from safetensors.torch import save_model
    rank, size = _tp_layout()
    os.makedirs(cache_dir, exist_ok=True)
    path = shard_cache_path(cache_dir, rank, size)
    tmp = path + f".tmp{os.getpid()}"
    save_model(model, tmp, metadata=_layout_meta(model, size))
    os.replace(tmp, path)  # atomic: a concurrently starting replica never sees a partial file
    return path


def load_shard(model: nn.Module, cache_dir: str) -> bool:
    """Load this rank's cached shard if it exists and matches the model's layout."""
    from safetensors import safe_open
    from safetensors.torch import load_model
    rank, size = _tp_layout()
    path = shard_cache_path(cache_dir, rank, size)
    if not os.path.isfile(path):
        return False
    try:
        with safe_open(path, framework="pt", device="cpu") as h:
            meta = h.metadata() or {}
        if meta != _layout_meta(model, size):
            return False
        load_model(model, path, strict=False, device=str(next(model.parameters()).device))
    except Exception:  # corrupt / foreign file: fall back to the checkpoint and rewrite it
        return False
    return True


def materialize(model: nn.Module, device, path: Optional[str] = None, subfolder: Optional[str] = None,
                seed: int = 0, convert: Optional[Callable] = None,
                shard_cache: Optional[str] = None) -> nn.Module:
    """Move to device and fill weights: this rank's cached shard if present, else the
    checkpoint under ``path`` (then cached), else deterministic random init."""
    model = model.to(device)
    shard_cache = shard_cache if shard_cache is not None else os.environ.get("SHAI_SHARD_CACHE") or None
    if shard_cache and subfolder:
        shard_cache = os.path.join(shard_cache, subfolder)
    files = find_safetensors(path, subfolder) if path else []
    if files and shard_cache and load_shard(model, shard_cache):
        model._shai_weights = "checkpoint"
        model._shai_shard_cache = "hit"
    elif files:
        load_into(model, load_safetensors(files), convert or getattr(model, "convert_hf_state_dict", None))
        model._shai_weights = "checkpoint"
        if shard_cache:
            save_shard(model, shard_cache)
            model._shai_shard_cache = "written"
    else:
        init_random_(model, seed)
        model._shai_weights = "random-init"
    model.eval()
    return model
