"""shai_amd.engines"""
import torch

_PRIMED: dict = {}  # device index -> the primer graph, kept alive: the generator frees its graph-safe
#                     state when the last registered graph is destroyed, and would re-create it in
#                     whatever mode the next capture runs in


def new_graph(device) -> "torch.cuda.CUDAGraph":
    """A fresh hipGraph (``torch.cuda.CUDAGraph``) for an engine's capture.

    The first capture on a device creates the CUDA generator's graph-safe RNG state tensors, and every later
    ``capture_begin`` fills them in place.  If that first capture runs under ``torch.inference_mode`` (the LLM
    engine does) they become inference tensors and a later capture outside it (the diffusion engines run
    under ``no_grad``) fails with "Inplace update to inference tensor outside InferenceMode".  Priming the
    state once with a one-op capture outside inference mode makes the captures order-independent."""
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _PRIMED:
        with torch.inference_mode(False), torch.cuda.device(idx):
            x = torch.zeros(1, device=f"cuda:{idx}")
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                x.add_(1)
            torch.cuda.synchronize(idx)
        _PRIMED[idx] = (g, x)
    return torch.cuda.CUDAGraph()
