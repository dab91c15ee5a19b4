"""Batched encoder engines: DistilBERT sentiment, ViT classification, YOLOS
detection, T5 embeddings.

The reference runs these one request at a time and ViT even reloads its model
per request (app/run-vit.py:40-41,48-49,60-61); here each model is resident on
the GPU and requests are batched by the server's EngineWorker.
"""
from __future__ import annotations

import base64
import io
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..tokenizers import load_tokenizer
from ..weights import materialize


def load_image(src: str):
    """URL / file path / data-URI / raw base64 -> PIL RGB.  (The GPU box has no
    network; http(s) URLs are fetched only when reachable.)"""
    from PIL import Image
    if src.startswith("data:"):
        raw = base64.b64decode(src.split(",", 1)[1])
        return Image.open(io.BytesIO(raw)).convert("RGB")
    if src.startswith("http://") or src.startswith("https://"):
        import requests
        r = requests.get(src, stream=True, timeout=10)
        r.raise_for_status()
        return Image.open(r.raw).convert("RGB")
    if src.startswith("file://"):
        src = src[7:]
    if os.path.exists(src):
        return Image.open(src).convert("RGB")
    raw = base64.b64decode(src)
    return Image.open(io.BytesIO(raw)).convert("RGB")


def synthetic_image(h=480, w=640, seed=0):
    """Deterministic test image (stand-in for the reference's COCO warm-up URL)."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    img = np.stack([(xx * 255 // w), (yy * 255 // h), rng.integers(0, 255, (h, w))], -1).astype(np.uint8)
    return Image.fromarray(img)


def _to_u8(img) -> torch.Tensor:
    return torch.from_numpy(np.asarray(img.convert("RGB"), dtype=np.uint8).copy())


class TextClassifierEngine:
    def __init__(self, cfg=None, device="cuda", model_path=None, seed=0):
        from ..models.bert import DistilBertConfig, DistilBertForSequenceClassification
        self.cfg = cfg or DistilBertConfig()
        self.device = torch.device(device)
        with torch.device(self.device):
            self.model = DistilBertForSequenceClassification(self.cfg)
        materialize(self.model, self.device, model_path, None, seed)
        c = self.cfg
        self.tokenizer = load_tokenizer(model_path, vocab_size=c.vocab_size, bos_id=c.cls_token_id,
                                        eos_id=c.sep_token_id, pad_id=c.pad_token_id, model_max_length=512)

    @torch.inference_mode()
    def classify(self, texts: Sequence[str]) -> List[str]:
        enc = self.tokenizer(list(texts), padding="longest", truncation=True, max_length=512, return_tensors="pt")
        ids = enc["input_ids"].to(self.device)
        mask = enc["attention_mask"].to(self.device)
        logits = self.model(ids, mask)
        return [self.cfg.id2label[int(i)] for i in logits.float().argmax(-1).tolist()]


class ImageClassifierEngine:
    """ViT classifier (run-vit.py).  Same-size batches run as one replayed HIP graph per batch size
    (uint8 NHWC in -> normalise -> encoder -> classifier), so a 12-layer ViT-base batch costs one launch."""

    def __init__(self, cfg=None, device="cuda", model_path=None, seed=0, labels=None, use_graphs=True):
        from ..models.vit import ViTConfig, ViTForImageClassification
        self.cfg = cfg or ViTConfig.vit_base()
        self.device = torch.device(device)
        with torch.device(self.device):
            self.model = ViTForImageClassification(self.cfg)
        materialize(self.model, self.device, model_path, None, seed)
        self.labels = labels or _load_labels(model_path) or {i: f"LABEL_{i}" for i in range(self.cfg.num_labels)}
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self._mean = torch.tensor(self.cfg.image_mean, device=self.device).view(1, 1, 1, 3)
        self._inv_std = 1.0 / torch.tensor(self.cfg.image_std, device=self.device).view(1, 1, 1, 3)
        self._graphs = {}

    def _forward_u8(self, x_u8: torch.Tensor) -> torch.Tensor:
        px = ((x_u8.float() * (1.0 / 255.0) - self._mean) * self._inv_std).to(torch.bfloat16)
        return self.model(px)

    @torch.inference_mode()
    def logits_u8(self, x_u8: torch.Tensor) -> torch.Tensor:
        """[B, H, W, 3] uint8 on the device at the model resolution -> logits [B, num_labels]."""
        B = x_u8.shape[0]
        if not self.use_graphs:
            return self._forward_u8(x_u8)
        g = self._graphs.get(B)
        if g is None:
            static = x_u8.clone()
            side = torch.cuda.Stream(device=self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                for _ in range(2):  # warm-up: GEMM autotuning and allocator growth happen outside capture
                    self._forward_u8(static)
            torch.cuda.current_stream(self.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = self._forward_u8(static)
            g = self._graphs[B] = (graph, static, out)
        graph, static, out = g
        static.copy_(x_u8)
        graph.replay()
        return out

    @torch.inference_mode()
    def warmup(self, max_batch: int) -> int:
        """Capture the HIP graph of every batch size 1 .. max_batch now (a serving replica's dynamic batcher
        forms any of them); returns how many graphs exist."""
        if self.use_graphs:
            H, W = self.cfg.image_size
            for b in range(1, max_batch + 1):
                self.logits_u8(torch.zeros(b, H, W, 3, dtype=torch.uint8, device=self.device))
        return len(self._graphs)

    @torch.inference_mode()
    def classify(self, images) -> List[str]:
        H, W = self.cfg.image_size
        x = torch.stack([_resize_u8(_to_u8(im) if not isinstance(im, torch.Tensor) else im, H, W)
                         for im in images]).to(self.device)
        logits = self.logits_u8(x)
        return [self.labels.get(int(i), str(int(i))) for i in logits.float().argmax(-1).tolist()]


class DetectorEngine:
    def __init__(self, cfg=None, device="cuda", model_path=None, seed=0, shortest_edge: Optional[int] = None,
                 threshold: float = 0.5):
        from ..models.vit import ViTConfig, YolosForObjectDetection
        self.cfg = cfg or ViTConfig.yolos_tiny()
        self.device = torch.device(device)
        with torch.device(self.device):
            self.model = YolosForObjectDetection(self.cfg)
        materialize(self.model, self.device, model_path, None, seed)
        self.labels = _load_labels(model_path) or {i: f"LABEL_{i}" for i in range(self.cfg.num_labels)}
        self.shortest_edge = shortest_edge or self.cfg.image_size[0]
        self.threshold = threshold

    def _target(self, h, w):
        s = self.shortest_edge / min(h, w)
        th, tw = int(round(h * s)), int(round(w * s))
        p = self.cfg.patch_size
        return max(p, th // p * p), max(p, tw // p * p)

    @torch.inference_mode()
    def detect(self, images) -> List[list]:
        from ..models.vit import YolosForObjectDetection, preprocess
        out = []
        for im in images:  # images differ in size: one forward each (tokens depend on the grid)
            u8 = _to_u8(im)
            h, w = u8.shape[:2]
            th, tw = self._target(h, w)
            px = preprocess(u8[None], (th, tw), self.cfg.image_mean, self.cfg.image_std, self.device)
            logits, boxes = self.model(px)
            out += YolosForObjectDetection.postprocess(logits, boxes, [(h, w)], self.threshold, self.labels)
        return out


class TextEmbeddingEngine:
    def __init__(self, cfg=None, device="cuda", model_path=None, seed=0):
        from ..models.t5 import T5Config, T5EncoderModel
        self.cfg = cfg or T5Config.v1_1_large()
        self.device = torch.device(device)
        with torch.device(self.device):
            self.model = T5EncoderModel(self.cfg)
        materialize(self.model, self.device, model_path, None, seed)
        self.tokenizer = load_tokenizer(model_path, vocab_size=self.cfg.vocab_size, bos_id=None,
                                        eos_id=self.cfg.eos_token_id, pad_id=self.cfg.pad_token_id,
                                        model_max_length=1024)

    @torch.inference_mode()
    def embed(self, texts: Sequence[str], max_length: int) -> np.ndarray:
        enc = self.tokenizer(list(texts), max_length=max_length, padding="max_length", truncation=True,
                             return_tensors="pt")
        ids = enc["input_ids"].to(self.device)
        mask = enc["attention_mask"].to(self.device)
        return self.model.encode_mean(ids, mask).cpu().numpy()


def _resize_u8(x: torch.Tensor, H: int, W: int) -> torch.Tensor:
    if x.shape[0] == H and x.shape[1] == W:
        return x
    t = x.permute(2, 0, 1)[None].float()
    t = torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=False, antialias=True)
    return t[0].permute(1, 2, 0).round().clamp(0, 255).to(torch.uint8)


def _load_labels(model_path):
    import json
    if model_path and os.path.exists(os.path.join(model_path, "config.json")):
        with open(os.path.join(model_path, "config.json")) as f:
            d = json.load(f)
        if "id2label" in d:
            return {int(k): v for k, v in d["id2label"].items()}
    return None
