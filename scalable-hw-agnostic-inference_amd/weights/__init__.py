"""Checkpoint loading: safetensors from a local directory (streamed, never
pickle), HF/diffusers key conversion per model, per-rank shard-on-load for
tensor parallel layers (TP layers slice rows/cols in their
``_load_from_state_dict`` hooks, so no pre-sharded files are needed), or
deterministic random init when no checkpoint is available (the offline GPU
box).  Replaces the reference's HF-Hub snapshot / ``parallel_model_load``
artifact flow (app/download_hf_model.py:1-8, app/t5_model_api.py:27-33).
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


def materialize(model: nn.Module, device, path: Optional[str] = None, subfolder: Optional[str] = None,
                seed: int = 0, convert: Optional[Callable] = None) -> nn.Module:
    """Move to device and fill weights: checkpoint if found under ``path`` else random init."""
    model = model.to(device)
    files = find_safetensors(path, subfolder) if path else []
    if files:
        load_into(model, load_safetensors(files), convert or getattr(model, "convert_hf_state_dict", None))
        model._shai_weights = "checkpoint"
    else:
        init_random_(model, seed)
        model._shai_weights = "random-init"
    model.eval()
    return model
